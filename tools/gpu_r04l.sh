#!/bin/bash
# round-4 call l: k_line_solve with the line cell indices requested two rows ahead (build_ab/c2.so;
# with 128-cell line pieces: build_ab/c2lm128.so) against the round-4 library (in-tree .so) and the
# 128-cell pieces alone (build_ab/lm128.so): C4 implicit steps, alternating, then kernel traces
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04l
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; grep '^{' "$OUT/$name.log" | tail -1 | cut -c1-300
  if [ $rc -ne 0 ]; then tail -c 700 "$OUT/$name.log"; echo "stopping after $name"; exit $rc; fi
}
B="tools/bench_implicit.py --case naca --steps 3 --warmup 1 --init-steps 5 --sweeps 1 --lines --operators assembled --second-from freestream"
for rep in 1 2; do
  run base_$rep 200 python3 -u $B
  for v in c2 lm128 c2lm128; do
    FVHIP_LIB=$(realpath fvens_amd/build_ab/$v.so) run ${v}_$rep 200 python3 -u $B
  done
done
for v in c2 c2lm128; do
  FVHIP_LIB=$(realpath fvens_amd/build_ab/$v.so) run tr_$v 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr_$v -o run -- python3 $B
done
run tr_base 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr_base -o run -- python3 $B
echo done
