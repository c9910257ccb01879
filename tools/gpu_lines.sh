#!/bin/bash
# GPU-box check of the line-implicit preconditioner: its tests, then the C4 implicit step with each
# library build given (FVHIP_LINE_MAX variants) and point-block Jacobi; every step under its own limit
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_implicit.py tests/test_gpu_viscous.py -m gpu -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/t_impl.log 2>&1; rc=$?; tail -n 3 gpurun_out/t_impl.log; [ $rc -le 1 ] || exit $rc
BI="tools/bench_implicit.py --case naca --steps 3 --warmup 1 --init-steps 5 --sweeps 1"
for lib in "$@"; do
  n=$(basename $lib .so)
  FVHIP_LIB=$(realpath $lib) timeout -k 10 300 python -u $BI --lines > gpurun_out/bi_$n.log 2>&1 || exit $?
  tail -n 2 gpurun_out/bi_$n.log | cut -c1-260
done
timeout -k 10 300 python -u $BI > gpurun_out/bi_pbj.log 2>&1 || exit $?
tail -n 2 gpurun_out/bi_pbj.log | cut -c1-260
