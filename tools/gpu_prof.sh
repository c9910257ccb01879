#!/bin/bash
# GPU-box profiling: rocprofv3 kernel trace + stats, then separate PMC passes (never combined with
# trace domains). Every step under its own time limit; stop at the first failure.
# usage: tools/gpu_prof.sh [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
ARGS="--steps 200 --warmup 20 --no-cpu-baseline --no-pipelined --no-implicit $*"
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -3 "$OUT/$name.log"
  [ $rc -eq 0 ] || { echo "stopping after $name"; exit $rc; }
}
run list 120 rocprofv3 -L
run trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS
run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS
run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS
run pmc_sq 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/sq -o run -- python3 bench.py $ARGS
run pmc_sq2 600 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq2 -o run -- python3 bench.py $ARGS
run pmc_lds 600 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_BRANCH --output-format csv -d $OUT/lds -o run -- python3 bench.py $ARGS
echo done
