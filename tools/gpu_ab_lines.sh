#!/bin/bash
# GPU-box A/B of library builds on the C4 line-implicit step (tools/bench_implicit.py, assembled operator):
#   tools/gpu_ab_lines.sh lib1.so lib2.so ...   (each run under its own time limit; stop at the first failure)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in ${AB_REPS:-1 2}; do
for lib in "$@"; do
  name=$(basename "$lib" .so)
  FVHIP_LIB=$(realpath "$lib") timeout -k 10 300 python tools/bench_implicit.py --case naca --steps 3 --warmup 1 \
    --init-steps 5 --sweeps 1 --lines --operators assembled,matrix-free > gpurun_out/abl_${name}_$rep.jsonl 2> gpurun_out/abl_${name}_$rep.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "rc=$rc"; tail -5 gpurun_out/abl_${name}_$rep.err; exit $rc; fi
  python3 -c "
import json
for l in open('gpurun_out/abl_${name}_$rep.jsonl'):
    d=json.loads(l); print('$name', d['operator'], d['ms_per_step'], d['lin_iters_per_step'], d['resratio'])
"
done
done
