#!/bin/bash
# round-4 probe call: implicit schedules (item 6), steady-state headline trace (item 3), Jacobian
# assembly trace + PMC passes (item 5). Each step under its own limit; stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04a
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -c 600 "$OUT/$name.log"; echo
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
}
run rccl_ranks 600 python3 -u -m pytest -v --timeout 500 --timeout-method thread tests/test_gpu_rccl_ranks.py -s
run newtests 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_tvdrk.py tests/test_gpu_implicit.py::test_partitioned_line_implicit_same_solution tests/test_gpu_implicit.py::test_partitioned_ilu_same_solution tests/test_gpu_implicit.py::test_one_backward_euler_step_matches_host tests/test_gpu_partition.py::test_partitioned_c5_eight_ranks -s
run jac 200 python3 -u tools/jac_probe.py --reps 100
for rep in 1 2; do
  FVHIP_LIB=$(realpath fvens_amd/build_ab/jl0.so) run jac_ab_jl0_$rep 200 python3 -u tools/jac_probe.py --reps 100
  run jac_ab_jl1_$rep 200 python3 -u tools/jac_probe.py --reps 100
done
run jac_trace 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/jtrace -o run -- python3 tools/jac_probe.py --reps 100
run jac_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/jfetch -o run -- python3 tools/jac_probe.py --reps 20
run jac_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/jwrite -o run -- python3 tools/jac_probe.py --reps 20
run jac_sq 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $OUT/jsq -o run -- python3 tools/jac_probe.py --reps 20
run steady_trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 2000 --warmup 20 --no-cpu-baseline --no-pipelined --no-implicit
run implicit_probe 500 python3 -u tools/implicit_probe.py
run plines 600 python3 -u tools/partitioned_lines_probe.py
run enqueue 400 python3 -u tools/enqueue_probe.py
run weno 400 python3 -u tools/weno_regression_probe.py --lambdas 20,0,1e-3,1
echo done
