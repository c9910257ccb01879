#!/bin/bash
# round-4 call c: multi-rank RCCL test, viscous parity after the per-row temperature terms, config-5 A/B,
# the driver's bench command; the hipGraph RCCL test last (its rank processes crashed in call b).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04c
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -c 600 "$OUT/$name.log"; echo
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
  if grep -q "returncode: -11\|(-11)\|(-6)\|(139)\|(134)" "$OUT/$name.log"; then echo "a child crashed in $name: stopping"; exit 7; fi
}
PYT="python3 -u -m pytest -v --timeout 600 --timeout-method thread -s"
run rccl_ranks 400 $PYT tests/test_gpu_rccl_ranks.py::test_rccl_ranks_on_one_gpu
run visc 900 $PYT tests/test_gpu_viscous.py tests/test_gpu_residual.py tests/test_gpu_partition.py -k "visc or plate or c5"
for rep in 1 2; do
  for v in jl0 vg1; do
    FVHIP_LIB=$(realpath fvens_amd/build_ab/$v.so) run c5_${v}_$rep 300 python3 -u bench.py --numerics config5 --steps 100 --warmup 10 --no-fast --no-pipelined --no-implicit --no-cpu-baseline
  done
  run c5_new_$rep 300 python3 -u bench.py --numerics config5 --steps 100 --warmup 10 --no-fast --no-pipelined --no-implicit --no-cpu-baseline
done
run bench_driver 600 python3 -u bench.py --steps 20 --warmup 5
run rccl_graph 400 $PYT tests/test_gpu_rccl_ranks.py::test_rccl_ranks_graph_on_one_gpu
echo done
