#!/bin/bash
# One gpurun call = a list of steps, each under its own time limit, stopped at the first failure.
#   bash tools/gpu_steps.sh OUTDIR [STEPFILE]        (steps from STEPFILE, else from stdin)
# A step line is "name timeout command ..." ('#' lines and blank lines skipped); its output goes to
# gpurun_out/OUTDIR/name.log. A step that exits with a status other than 0 or 1 (pytest failures are
# 1), a time limit (124/137) or a child that crashed (-11/-6/139/134 in its log) ends the call: no
# further GPU step runs after a fault, an abort or a hang.
# (The per-call scripts of rounds 1-4, tools/gpu_*.sh, are in git history before round 5.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p "$OUT"
STEPS=$(if [ $# -ge 2 ]; then cat "$2"; else cat; fi)
while IFS= read -r line; do
  case "$line" in ''|'#'*) continue ;; esac
  name=${line%% *}; rest=${line#* }
  to=${rest%% *}; cmd=${rest#* }
  echo "== $name ($to s): $cmd"; date
  timeout -k 10 "$to" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "rc=$rc"; tail -c 600 "$OUT/$name.log"; echo
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
  if grep -q "returncode: -11\|(-11)\|(-6)\|(139)\|(134)\|Segmentation fault" "$OUT/$name.log"; then
    echo "a child crashed in $name: stopping"; exit 7
  fi
done <<< "$STEPS"
echo "all steps done"
