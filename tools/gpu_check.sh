#!/bin/bash
# GPU-box runner: each GPU step under its own time limit; stop at the first crash/timeout
# (exit codes other than 0/1 = pytest test failures).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" ; date
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    smoke) step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) step pytest_gpu 1100 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ;;
    jtests) step pytest_jac 900 python -u -m pytest tests/test_gpu_jacobian.py -m gpu -q -rf -x ;;
    bench) step bench 600 python -u bench.py ;;
    benchd) step bench_driver 600 python -u bench.py --steps 20 --warmup 5 ;;
    benchq) step bench 600 python bench.py --steps 20 --warmup 3 ;;
    prof) step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline ;;
  esac
done
