set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_implicit.py -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/pyt_impl.log 2>&1; rc=$?; tail -5 gpurun_out/pyt_impl.log; [ $rc -eq 0 ] || exit $rc
for a in "--sweeps 1 --lines" "--sweeps 1 --ilu" "--sweeps 1" ; do
  timeout -k 10 300 python -u tools/bench_implicit.py --case naca --steps 3 --warmup 1 --init-steps 5 --operators assembled $a >> gpurun_out/impl_cmp.jsonl 2>> gpurun_out/impl_cmp.err || exit $?
done
cat gpurun_out/impl_cmp.jsonl
