#!/bin/bash
# round-4 call b: multi-rank RCCL test, new/changed GPU tests, config-5 A/B (per-slot viscous geometry),
# long implicit schedules. Test failures (rc 1) do not stop the call; crashes and timeouts do.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04b
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -c 800 "$OUT/$name.log"; echo
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
}
PYT="python3 -u -m pytest -v --timeout 600 --timeout-method thread -s"
run rccl_ranks 600 $PYT tests/test_gpu_rccl_ranks.py
run newtests 900 $PYT tests/test_gpu_implicit.py::test_partitioned_line_implicit_same_solution tests/test_gpu_implicit.py::test_naca0012_weno_implicit_functional_regression tests/test_gpu_partition.py::test_partitioned_c5_eight_ranks
run jacvisc 900 $PYT tests/test_gpu_jacobian.py tests/test_gpu_viscous.py tests/test_gpu_residual.py
for rep in 1 2; do
  FVHIP_LIB=$(realpath fvens_amd/build_ab/jl0.so) run c5_old_$rep 300 python3 -u bench.py --numerics config5 --steps 100 --warmup 10 --no-fast --no-pipelined --no-implicit --no-cpu-baseline
  run c5_new_$rep 300 python3 -u bench.py --numerics config5 --steps 100 --warmup 10 --no-fast --no-pipelined --no-implicit --no-cpu-baseline
done
run implicit_long 600 python3 -u tools/implicit_probe.py --schedules 20:25:25:150:25:25,20:25:25:150:10:10,40:10:10:150:25:25
echo done
