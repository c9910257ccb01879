#!/bin/bash
# round-4 call s: block-Jacobi apply and multicolour Gauss-Seidel with four lanes per cell (in-tree) against
# the lane-per-cell kernels (build_ab/rows0.so): implicit states bitwise (dumps kept under /tmp on the box),
# the Jacobian / implicit GPU tests, and C4 implicit steps with point-block Jacobi (4 sweeps) timed
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04s
mkdir -p $OUT
D=$(mktemp -d)
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -c 500 "$OUT/$name.log"; echo
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
OLD=$(realpath fvens_amd/build_ab/rows0.so)
run dump_new 200 python3 -u tools/implicit_state_dump.py $D/new.npz
FVHIP_LIB=$OLD run dump_old 200 python3 -u tools/implicit_state_dump.py $D/old.npz
run compare 60 python3 -c "
import numpy as np
a=np.load('$D/new.npz'); b=np.load('$D/old.npz')
for k in a.files: print(k, 'bitwise' if np.array_equal(a[k], b[k]) else 'DIFFERENT', float(np.abs(a[k]-b[k]).max()))
assert all(np.array_equal(a[k], b[k]) for k in a.files)
"
rm -rf $D
run tests 600 python3 -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_jacobian.py tests/test_gpu_implicit.py tests/test_gpu_driver.py tests/test_gpu_partition.py
B="tools/bench_implicit.py --case naca --steps 3 --warmup 1 --init-steps 5 --sweeps 2 --gs --operators assembled --second-from freestream"
for rep in 1 2; do
  run new_$rep 200 python3 -u $B
  FVHIP_LIB=$OLD run old_$rep 200 python3 -u $B
done
run tr_new 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr_new -o run -- python3 $B
FVHIP_LIB=$OLD run tr_old 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr_old -o run -- python3 $B
echo done
