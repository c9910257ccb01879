#!/bin/bash
# round-4 call v: the round-2 full-size convergence run of the bench's C4 mesh repeated on the round-4 code
# (first-order LLF, line-implicit, GMRES(40), expResidualRamp CFL 5 -> 1000, to a 1e-6 drop from the peak)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04v
mkdir -p $OUT
timeout -k 10 1000 python3 -u tools/c4_converge_chunked.py --init-flux LLF --wall 1e-5 --init-steps 6000 --init-drop 1e-6 --main-steps 0 --seconds 640 --lines --cfl 5 1000 > $OUT/conv.log 2>&1
rc=$?
tail -5 $OUT/conv.log
exit $rc
