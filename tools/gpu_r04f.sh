#!/bin/bash
# round-4 call f: RCCL ranks with config-4/5 numerics, the 2-rank bench rehearsals, an implicit-step trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04f
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -c 700 "$OUT/$name.log"; echo
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
  if grep -q "returncode: -11\|(-11)\|(-6)\|(139)\|(134)" "$OUT/$name.log"; then echo "a child crashed in $name: stopping"; exit 7; fi
}
run rccl_ranks 500 python3 -u -m pytest -v --timeout 300 --timeout-method thread -s tests/test_gpu_rccl_ranks.py::test_rccl_ranks_on_one_gpu
run bench_ranks 700 python3 -u -m pytest -v --timeout 330 --timeout-method thread -s tests/test_gpu_bench_ranks.py
run implicit_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/itrace -o run -- python3 tools/bench_implicit.py --case naca --steps 3 --warmup 1 --init-steps 5 --sweeps 1 --lines --operators assembled
echo done
