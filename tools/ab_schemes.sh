#!/bin/bash
# GPU-box A/B of library builds on the scheme benchmark (one residual with local time steps):
#   tools/ab_schemes.sh CASES lib1.so lib2.so ...   (CASES: comma-separated bench_schemes case names)
# each run under its own time limit; stop at the first crash/timeout
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cases=$1; shift
for rep in ${AB_REPS:-1 2}; do
for lib in "$@"; do
  name=$(basename "$lib" .so)
  echo "== $name rep $rep"
  FVHIP_LIB=$(realpath "$lib") timeout -k 10 300 python tools/bench_schemes.py --only "$cases" --warmup 600 --steps 300 \
    > gpurun_out/abs_${name}_$rep.jsonl 2> gpurun_out/abs_${name}_$rep.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "rc=$rc"; tail -5 gpurun_out/abs_${name}_$rep.err; exit $rc; fi
  python3 -c "
import json
for l in open('gpurun_out/abs_${name}_$rep.jsonl'):
    d=json.loads(l); print('$name', d.get('case'), d.get('ms_per_residual'), d.get('kernels_ms'))
"
done
done
