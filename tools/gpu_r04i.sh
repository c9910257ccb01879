#!/bin/bash
# round-4 call i: patch size A/B for the small BASELINE meshes (FVHIP_PATCH_SLOTS: faces per patch the
# layout aims at; the kernel's blocks stay 256 threads), config 2 (C2) and config 3 (flat plate), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04i
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; grep -o '"kernels_ms": {[^}]*}' "$OUT/$name.log" | tail -1
  if [ $rc -ne 0 ]; then tail -c 700 "$OUT/$name.log"; echo "stopping after $name"; exit $rc; fi
}
A="--steps 300 --warmup 20 --no-cpu-baseline --no-implicit --no-fast --no-pipelined"
for rep in 1 2; do
  for cap in 256 192 160 128; do
    FVHIP_PATCH_SLOTS=$cap run c2_${cap}_$rep 200 python3 -u bench.py --numerics config2 $A
  done
  for cap in 256 192 160; do
    FVHIP_PATCH_SLOTS=$cap run c3_${cap}_$rep 200 python3 -u bench.py --numerics config3 $A
  done
  for cap in 256 224; do
    FVHIP_PATCH_SLOTS=$cap run c4_${cap}_$rep 200 python3 -u bench.py $A
  done
done
echo done
bash tools/gpu_r04j.sh
