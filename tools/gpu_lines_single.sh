#!/bin/bash
# GPU-box: implicit tests, then the C4 line-implicit step with fp64 and fp32 line factors (prec_single),
# alternating, and a kernel trace of the fp32 variant; each step under its own time limit
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_implicit.py -q -x --timeout 300 --timeout-method thread > gpurun_out/pyt_impl.log 2>&1
rc=$?; tail -3 gpurun_out/pyt_impl.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in fp64 fp32; do
    extra=""; [ $v = fp32 ] && extra="--prec-single"
    timeout -k 10 300 python tools/bench_implicit.py --case naca --steps 3 --warmup 1 --init-steps 5 --sweeps 1 --lines \
      --operators assembled,matrix-free $extra > gpurun_out/abl_${v}_$rep.jsonl 2> gpurun_out/abl_${v}_$rep.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/abl_${v}_$rep.err; exit $rc; }
    python3 -c "
import json
for l in open('gpurun_out/abl_${v}_$rep.jsonl'):
    d=json.loads(l); print('$v', d['operator'], d['ms_per_step'], d['lin_iters_per_step'], d['resratio'])
"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lines -o run -- python3 tools/bench_implicit.py \
  --case naca --steps 3 --warmup 1 --init-steps 5 --sweeps 1 --lines --prec-single --operators assembled > gpurun_out/prof_lines.log 2>&1
echo "prof rc=$?"
