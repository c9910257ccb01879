#!/bin/bash
# round-4 call o: the line-implicit preconditioner's blocks in fp32 (prec_single; arithmetic in fp64) against
# fp64 storage: C4 (assembled), C5 laminar (assembled), flat plate (matrix-free), alternating
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04o
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; grep '^{' "$OUT/$name.log" | tail -1 | cut -c1-260
  if [ $rc -ne 0 ]; then tail -c 700 "$OUT/$name.log"; echo "stopping after $name"; exit $rc; fi
}
for rep in 1 2; do
  for sp in "" "--prec-single"; do
    t=${sp:+single}; t=${t:-double}
    run naca_${t}_$rep 200 python3 -u tools/bench_implicit.py --case naca --steps 3 --warmup 1 --init-steps 5 --sweeps 1 --lines --operators assembled --second-from freestream $sp
    run c5_${t}_$rep 300 python3 -u tools/bench_implicit.py --case visc-c5 --steps 3 --warmup 1 --init-steps 5 --sweeps 1 --lines --operators assembled --second-from freestream $sp
    run plate_${t}_$rep 200 python3 -u tools/bench_implicit.py --case plate --steps 3 --warmup 1 --init-steps 5 --sweeps 1 --lines --operators matrix-free --second-from start $sp
  done
done
echo done
