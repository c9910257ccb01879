#!/bin/bash
# GPU-box PMC passes beyond tools/gpu_prof.sh: the VALU instruction mix and lane activity of the
# headline fused kernel (bench.py), and trace + traffic + VALU passes of the viscous and limited
# fused instantiations (tools/bench_schemes.py). Each pass its own run, no trace domains with --pmc;
# every step under its own time limit; stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"; date
  mkdir -p gpurun_out/logs
  timeout -k 10 "$to" "$@" > "gpurun_out/logs/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 2 "gpurun_out/logs/$name.log"
  [ $rc -eq 0 ] || { echo "stopping after $name"; exit $rc; }
}
B="python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-pipelined --no-implicit --no-fast"
VMIX="SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT"
VLANE="SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
O=gpurun_out/pvalu
run vmix 150 rocprofv3 --pmc $VMIX --output-format csv -d $O/vmix -o run -- $B
run vlane 150 rocprofv3 --pmc $VLANE --output-format csv -d $O/vlane -o run -- $B
S="python3 tools/bench_schemes.py --steps 50 --warmup 10 --only roe-wls-muscl-viscous,roe-wls-venkatakrishnan,plate-hllc-wls-viscous"
O=gpurun_out/pschemes
run s_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $S
run s_fetch 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $S
run s_write 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $S
run s_vmix 150 rocprofv3 --pmc $VMIX --output-format csv -d $O/vmix -o run -- $S
run s_vlane 150 rocprofv3 --pmc $VLANE --output-format csv -d $O/vlane -o run -- $S
echo done
