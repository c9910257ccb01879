#!/bin/bash
# GPU-box: the whole GPU suite, then the driver's bench command for BASELINE configs 4 and 5 on one GPU
# (bench.py --numerics config4 / config5); each step under its own time limit, stop at the first failure
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --numerics config4 --steps 20 --warmup 5 > gpurun_out/bench_c4.log 2>&1
rc=$?; tail -c 400 gpurun_out/bench_c4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --numerics config5 --steps 20 --warmup 5 --no-pipelined > gpurun_out/bench_c5.log 2>&1
rc=$?; tail -c 400 gpurun_out/bench_c5.log; exit $rc
