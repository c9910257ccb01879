#!/bin/bash
# Diagnostic: the hipGraph-captured RCCL rank step (fvhip_set_residual_graph) on 2 ranks of one GPU, each
# rank's full output (RCCL INFO log, the native crash report of tools/probes/crashtrace.c) in its own file.
# usage: bash tools/probes/graph_capture_probe.sh OUTDIR
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=$1
mkdir -p "$OUT"
gcc -shared -fPIC -O1 -g -o tools/bin/libcrashtrace.so tools/probes/crashtrace.c || exit 3
PORT=$(python3 -c "import socket; s=socket.socket(); s.bind(('127.0.0.1',0)); print(s.getsockname()[1])")
pids=()
for r in 0 1; do
  RANK=$r LOCAL_RANK=0 WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT NCCL_HOSTID=fvhip-rank-$r \
  NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,P2P,NET,PROXY,COLL,ENV \
  FVHIP_CRASHTRACE=$PWD/tools/bin/libcrashtrace.so \
  timeout -k 5 150 python3 -u tests/rccl_rank_worker.py /tmp/graph_r$r.json naca_small graph graph > "$OUT/rank$r.log" 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=$?; done
echo "ranks done, last status $rc"
for r in 0 1; do echo "--- rank $r"; grep -n "crashtrace\|\[rank\|WARN\|rror" "$OUT/rank$r.log" | head -40; done
exit 0
