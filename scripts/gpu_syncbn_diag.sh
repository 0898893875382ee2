#!/bin/bash
# SyncBN 2-rank worker run directly (streamed progress), to time / diagnose tests/test_gpu_syncbn.py.
# Cases: "NET_FUNCTION SYNC_BN" pairs (CASES="1 1" runs one); each 3 steps under its own 100 s limit.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 OMP_NUM_THREADS=2 SYNCBN_VERBOSE=1
L=gpurun_out/syncbn_diag.log
: > $L
port=29400
if [ -n "$CASES" ]; then set -- "$CASES"; else set -- "0 1" "1 0" "1 1"; fi
for c in "$@"; do
  set -- $c
  port=$((port + 1))
  echo "=== NET_FUNCTION=$1 SYNC_BN=$2 STEPS=${STEPS:-3} $(date +%T)" >> $L
  KATIB_DARTS_NET_FUNCTION=$1 SYNC_BN=$2 STEPS=${STEPS:-3} timeout -k 10 100 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port tests/gpu_syncbn_worker.py 2>&1 | grep -v "Gloo\|socket.cpp\|amdgpu.ids" >> $L
  rc=$?
  echo "[rc=$rc] $(date +%T)" >> $L
  case $rc in 134|139) exit $rc ;; esac
done
