#!/bin/bash
# round-4 call y: BASELINE config 5's implicit figure with the matrix-free operator (as the config states)
# beside the assembled one, from the free stream and after the first-order start
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04y
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; grep '^{' "$OUT/$name.log" | cut -c1-330; echo
  if [ $rc -ne 0 ]; then tail -c 500 "$OUT/$name.log"; echo "stopping after $name"; exit $rc; fi
}
run c5_free 400 python3 -u tools/bench_implicit.py --case visc-c5 --steps 3 --warmup 1 --init-steps 5 --sweeps 1 --lines --operators assembled,matrix-free --second-from freestream
echo done
