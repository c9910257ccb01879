#!/bin/bash
# round-4 call e: phase probes of the config-4 (Venkatakrishnan) and config-5 (viscous) fused kernels:
# the full kernel and builds without the gradient phase, without the faces, staging + sums only, without
# the limiter / the viscous term (tools/gpu_r04e.sh; results per line: kernel ms of the probe build)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04e
mkdir -p $OUT
ARGS="--steps 100 --warmup 10 --no-fast --no-pipelined --no-implicit --no-cpu-baseline --preheat-ms 300"
one() {  # name lib numerics
  local name=$1 lib=$2 num=$3
  FVHIP_LIB=$(realpath $lib) timeout -k 10 300 python3 -u bench.py --numerics $num $ARGS > $OUT/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -5 $OUT/$name.log; exit $rc; fi
  python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/$name.log') if l.startswith('{')][-1]
print('$name', '$num', d['kernels_ms'], d['roofline']['frac'])
"
}
for rep in 1 2; do
  for num in config4 config5; do
    one full_${num}_$rep fvens_amd/libfvhip.so $num
    for v in nograd noface stage; do one ${v}_${num}_$rep fvens_amd/build_ab/pr_$v.so $num; done
  done
  one nolim_config4_$rep fvens_amd/build_ab/pr_nolim.so config4
  one novisc_config5_$rep fvens_amd/build_ab/pr_novisc.so config5
done
echo done
