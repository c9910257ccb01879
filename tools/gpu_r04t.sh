#!/bin/bash
# round-4 call t (final tree): multi-rank RCCL test, the whole GPU suite, smoke, the headline's rocprofv3
# trace and PMC passes (each its own run), the driver's bench command twice, configs 3/4/5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04t
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -c 400 "$OUT/$name.log"; echo
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
  if grep -q "returncode: -11\|(-11)\|(-6)\|(139)\|(134)" "$OUT/$name.log"; then echo "a child crashed in $name: stopping"; exit 7; fi
}
run rccl_ranks 400 python3 -u -m pytest -v --timeout 300 --timeout-method thread -s tests/test_gpu_rccl_ranks.py::test_rccl_ranks_on_one_gpu
run suite 1000 python3 -u -m pytest tests -m gpu -q -rf --timeout 450 --timeout-method thread -k "not rccl_ranks_on_one_gpu"
run smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()"
A="--steps 200 --warmup 20 --no-cpu-baseline --no-pipelined --no-implicit"
run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof/trace -o run -- python3 bench.py $A
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/prof/fetch -o run -- python3 bench.py $A
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/prof/write -o run -- python3 bench.py $A
run pmc_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/prof/sq -o run -- python3 bench.py $A
run pmc_sq2 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/prof/sq2 -o run -- python3 bench.py $A
run bench_driver_1 400 python3 -u bench.py --steps 20 --warmup 5
run config4 400 python3 -u bench.py --numerics config4 --steps 100 --warmup 10
run config5 500 python3 -u bench.py --numerics config5 --steps 100 --warmup 10
run config3 400 python3 -u bench.py --numerics config3 --steps 100 --warmup 10
run bench_driver_2 400 python3 -u bench.py --steps 20 --warmup 5
echo done
