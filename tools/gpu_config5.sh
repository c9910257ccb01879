#!/bin/bash
# GPU-box: partition tests, then BASELINE config 5 (C5 mesh, laminar viscous) through bench.py on one GPU
# and the single-GPU multi-rank proxy of C5 split 8 ways; each step under its own time limit
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_partition.py -q -x --timeout 300 --timeout-method thread > gpurun_out/pyt_part.log 2>&1
rc=$?; tail -3 gpurun_out/pyt_part.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --numerics config5 --steps 20 --warmup 5 --no-pipelined > gpurun_out/bench_c5.log 2>&1
rc=$?; tail -c 600 gpurun_out/bench_c5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u tools/scale_proxy.py --config5 --parts 8 > gpurun_out/scale_proxy_c5.jsonl 2> gpurun_out/scale_proxy_c5.err
rc=$?; echo "proxy rc=$rc"; exit $rc
