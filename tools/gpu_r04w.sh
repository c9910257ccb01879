#!/bin/bash
# round-4 call w: the round-2 convergence run of the full C4 at 1e-3 wall spacing repeated on the round-4 code
# (first-order Roe, point-block Jacobi, GMRES(40), expResidualRamp CFL 5 -> 200, to a 1e-6 drop from the peak)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04w
mkdir -p $OUT
timeout -k 10 1000 python3 -u tools/c4_converge_chunked.py --init-flux ROE --wall 1e-3 --init-steps 9500 --init-drop 1e-6 --main-steps 0 --seconds 900 > $OUT/conv.log 2>&1
rc=$?
tail -5 $OUT/conv.log
exit $rc
