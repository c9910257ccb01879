#!/bin/bash
# GPU-box A/B of library builds on the bench workload: tools/gpu_ab.sh lib1.so lib2.so ...
# (each run under its own time limit; stop at the first crash/timeout)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ARGS=${AB_ARGS:-"--steps 200 --warmup 20 --no-fast --no-pipelined --no-implicit --no-cpu-baseline"}
for lib in "$@"; do
  name=$(basename "$lib" .so)
  echo "== $name"
  FVHIP_LIB=$(realpath "$lib") timeout -k 10 300 python bench.py $ARGS > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "rc=$rc"; tail -5 gpurun_out/ab_$name.err; exit $rc; fi
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/ab_$name.json').read().strip().splitlines()[-1])
print('$name', 'ms/step', d['ms_per_step'], 'kernels', d['kernels_ms'], 'staged', d['staged_path']['kernels_ms'])
"
done
