#!/bin/bash
# round-4 call g: smoke, bench lines for BASELINE configs 2 and 3 (new --numerics), the driver's bench
# command, and the PMC passes of the config-3 fused kernel (each pass its own run, no trace domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04g
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -c 700 "$OUT/$name.log"; echo
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
run smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()"
run config3 400 python3 -u bench.py --numerics config3 --steps 100 --warmup 10
run config2 300 python3 -u bench.py --numerics config2 --steps 100 --warmup 10
run bench_driver 400 python3 -u bench.py --steps 20 --warmup 5
run iprobe 300 python3 -u tools/implicit_probe.py --schedules "0:25:25:6:25:25,0:25:25:6:10:10,3:25:25:6:25:25"
run bimp_free 300 python3 -u tools/bench_implicit.py --case naca --steps 3 --warmup 1 --init-steps 5 --sweeps 1 --lines --operators assembled --second-from freestream
A3="--numerics config3 --steps 100 --warmup 10 --no-cpu-baseline --no-pipelined --no-implicit"
run c3_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3/trace -o run -- python3 bench.py $A3
run c3_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/c3/fetch -o run -- python3 bench.py $A3
run c3_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/c3/write -o run -- python3 bench.py $A3
run c3_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/c3/sq -o run -- python3 bench.py $A3
run c3_sq2 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/c3/sq2 -o run -- python3 bench.py $A3
echo done
