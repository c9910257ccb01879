#!/bin/bash
# round-4 call u (final tree): multi-rank RCCL test, the whole GPU suite, smoke, the driver's bench command
# twice, configs 2-5 (BASELINE configurations, one line each)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04u
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -c 300 "$OUT/$name.log"; echo
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
  if grep -q "returncode: -11\|(-11)\|(-6)\|(139)\|(134)" "$OUT/$name.log"; then echo "a child crashed in $name: stopping"; exit 7; fi
}
run rccl_ranks 400 python3 -u -m pytest -v --timeout 300 --timeout-method thread -s tests/test_gpu_rccl_ranks.py::test_rccl_ranks_on_one_gpu
run suite 1000 python3 -u -m pytest tests -m gpu -q -rf --timeout 450 --timeout-method thread -k "not rccl_ranks_on_one_gpu"
run smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()"
run bench_driver_1 400 python3 -u bench.py --steps 20 --warmup 5
run config2 300 python3 -u bench.py --numerics config2 --steps 100 --warmup 10
run config3 400 python3 -u bench.py --numerics config3 --steps 100 --warmup 10
run config4 400 python3 -u bench.py --numerics config4 --steps 100 --warmup 10
run config5 500 python3 -u bench.py --numerics config5 --steps 100 --warmup 10
run bench_driver_2 400 python3 -u bench.py --steps 20 --warmup 5
echo done
