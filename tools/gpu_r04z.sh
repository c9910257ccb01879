#!/bin/bash
# round-4 call z: bench.py --numerics config5 with its matrix-free implicit figure, and the bench GPU tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04z
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -c 400 "$OUT/$name.log"; echo
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
run config5 500 python3 -u bench.py --numerics config5 --steps 100 --warmup 10
run bench_tests 900 python3 -u -m pytest -q -x --timeout 450 --timeout-method thread tests/test_gpu_bench_ranks.py
echo done
