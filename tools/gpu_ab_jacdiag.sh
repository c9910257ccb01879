set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
for v in jd0 jd1; do
  FVHIP_LIB=$(realpath fvens_amd/build_ab/$v.so) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_${v}_$rep -o run -- python3 tools/bench_implicit.py --case naca --steps 3 --warmup 1 --init-steps 5 --sweeps 1 --lines --operators assembled > gpurun_out/p_${v}_$rep.log 2>&1 || { echo "fail $v"; tail -5 gpurun_out/p_${v}_$rep.log; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/p_${v}_$rep/run_kernel_stats.csv')):
    if 'jac_diag' in r['Name'] or 'block_apply' in r['Name']: print('$v', r['Name'][:22], r['Calls'], r['AverageNs'])
"
done
done
