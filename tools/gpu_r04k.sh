#!/bin/bash
# round-4 call k: the C4 line set (tools/line_probe.py) and PMC of the implicit step's kernels (FETCH /
# WRITE / SQ in separate passes over tools/bench_implicit.py, summarised by tools/pmc_summary.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04k
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; grep '^{' "$OUT/$name.log" | tail -1 | cut -c1-1500
  if [ $rc -ne 0 ]; then tail -c 700 "$OUT/$name.log"; echo "stopping after $name"; exit $rc; fi
}
run lines 200 python3 -u tools/line_probe.py
B="tools/bench_implicit.py --case naca --steps 3 --warmup 1 --init-steps 5 --sweeps 1 --lines --operators assembled --second-from freestream"
run itrace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/imp/trace -o run -- python3 $B
run ifetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/imp/fetch -o run -- python3 $B
run iwrite 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/imp/write -o run -- python3 $B
run isq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/imp/sq -o run -- python3 $B
run isq2 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/imp/sq2 -o run -- python3 $B
echo done
