#!/bin/bash
# round-4 call n: host-pointer entries reordering on the device (one contiguous transfer each way, k_gather /
# k_scatter) -- the whole GPU suite on the new library, then the bench's host_boundary figure (PCIe-inclusive
# fvhip_compute_residual) for the new library and the previous one (build_ab/hostold.so), alternating
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04n
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; grep -o '"host_boundary": {[^}]*}' "$OUT/$name.log" | tail -1; tail -c 300 "$OUT/$name.log"; echo
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
  if grep -q "returncode: -11\|(-11)\|(-6)\|(139)\|(134)" "$OUT/$name.log"; then echo "a child crashed in $name: stopping"; exit 7; fi
}
run suite 1000 python3 -u -m pytest tests -m gpu -q -rf --timeout 450 --timeout-method thread -k "not rccl_ranks_on_one_gpu"
run rccl_ranks 400 python3 -u -m pytest -v --timeout 300 --timeout-method thread -s tests/test_gpu_rccl_ranks.py::test_rccl_ranks_on_one_gpu
A="--steps 50 --warmup 5 --no-cpu-baseline --no-implicit --no-fast --no-pipelined"
for rep in 1 2; do
  run host_new_$rep 300 python3 -u bench.py $A
  FVHIP_LIB=$(realpath fvens_amd/build_ab/hostold.so) run host_old_$rep 300 python3 -u bench.py $A
done
echo done
