#!/bin/bash
# round-4 call aa: the fused residual compiled with LLVM's max-ilp and max-memory-clause machine schedulers
# (build_ab/*.so, -mllvm --amdgpu-sched-strategy=...) against the default: C4 bitwise parity test for each,
# then headline / config 4 / config 5 kernel times, alternating
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04aa
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; grep -o '"kernels_ms": {[^}]*}' "$OUT/$name.log" | head -1; tail -c 200 "$OUT/$name.log"; echo
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
for v in max-ilp max-memory-clause; do
  FVHIP_LIB=$(realpath fvens_amd/build_ab/$v.so) run parity_$v 400 python3 -u -m pytest -q -x --timeout 300 --timeout-method thread "tests/test_gpu_fullsize.py::test_c4_residual_bitwise"
done
A="--steps 300 --warmup 20 --no-cpu-baseline --no-implicit --no-fast --no-pipelined"
for rep in 1 2; do
  for num in headline config4 config5; do
    run ${num}_base_$rep 300 python3 -u bench.py --numerics $num $A
    for v in max-ilp max-memory-clause; do
      FVHIP_LIB=$(realpath fvens_amd/build_ab/$v.so) run ${num}_${v}_$rep 300 python3 -u bench.py --numerics $num $A
    done
  done
done
echo done
