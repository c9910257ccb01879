set -u
cd ${GRAFT_REPO_ROOT}
O="--only roe-wls-muscl-viscous,plate-hllc-wls-viscous,roe-wls-muscl"
timeout -k 10 200 python tools/bench_schemes.py $O > gpurun_out/vis_A.jsonl 2>/dev/null || exit 3
timeout -k 10 200 python tools/bench_schemes.py $O --staged > gpurun_out/vis_S.jsonl 2>/dev/null || exit 3
FVHIP_LIB=$PWD/fvens_amd/libfvhip_vB.so timeout -k 10 200 python tools/bench_schemes.py $O > gpurun_out/vis_B.jsonl 2>/dev/null || exit 3
cat gpurun_out/vis_A.jsonl gpurun_out/vis_S.jsonl gpurun_out/vis_B.jsonl | cut -c1-330
