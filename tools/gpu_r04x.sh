#!/bin/bash
# round-4 call x (final tree): the driver's bench command and a 2,000-step rocprofv3 kernel trace of the same
# headline on one box, so the committed --stats average and the bench line's kernel time come from the same GPU
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04x
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -c 300 "$OUT/$name.log"; echo
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
run bench_driver 400 python3 -u bench.py --steps 20 --warmup 5
run steady_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 2000 --warmup 20 --no-cpu-baseline --no-pipelined --no-implicit
rm -f $OUT/trace/run_kernel_trace.csv.gz
echo done
