#!/bin/bash
# GPU-box runs of tools/c4_converge.py (first-order stage) with the line-implicit preconditioner
# usage: tools/c4_lines.sh SCALE STEPS "label:args" ... ; every run under its own time limit
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
S=$1; N=$2; shift 2
for spec in "$@"; do
  label=${spec%%:*}; args=${spec#*:}
  echo "== $label ($args)"
  timeout -k 10 ${RUN_LIMIT:-300} python -u tools/c4_converge.py --scale $S --init-steps $N --main-steps 0 --init-tol 1e-7 $args > gpurun_out/c4l_$label.log 2>&1
  rc=$?
  grep -E '^init' gpurun_out/c4l_$label.log | cut -c1-600
  if [ $rc -ne 0 ]; then echo "rc=$rc"; tail -3 gpurun_out/c4l_$label.log; [ $rc -ne 1 ] && exit $rc; fi
done
