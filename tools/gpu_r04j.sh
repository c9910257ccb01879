#!/bin/bash
# round-4 call j: line-implicit preconditioner with shorter line pieces (FVHIP_LINE_MAX 256 = default,
# 128, 64, 32; builds fvens_amd/build_ab/lm*.so): C4 implicit steps (time per step, GMRES iterations,
# residual ratio), alternating, and a kernel trace of the default and the 64-cell pieces.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04j
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; grep '^{' "$OUT/$name.log" | tail -1 | cut -c1-400
  if [ $rc -ne 0 ]; then tail -c 700 "$OUT/$name.log"; echo "stopping after $name"; exit $rc; fi
}
B="tools/bench_implicit.py --case naca --steps 3 --warmup 1 --init-steps 5 --sweeps 1 --lines --operators assembled,matrix-free --second-from freestream"
for rep in 1 2; do
  run lm256_$rep 200 python3 -u $B
  for v in 128 64 32; do
    FVHIP_LIB=$(realpath fvens_amd/build_ab/lm$v.so) run lm${v}_$rep 200 python3 -u $B
  done
done
run tr256 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr256 -o run -- python3 $B
FVHIP_LIB=$(realpath fvens_amd/build_ab/lm64.so) run tr64 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr64 -o run -- python3 $B
echo done
