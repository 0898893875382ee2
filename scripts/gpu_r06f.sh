#!/bin/bash
# fold_sync single-workgroup small-payload path: xGMI / SyncBN numerics (2 ranks sharing the GPU), then the
# 2- and 4-rank SyncBN B5 step (shared GPU: the rendezvous path, not a scaling number).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$(pwd)
L=gpurun_out/r06f.log
: > $L
timeout -k 10 600 python -u -m pytest tests/test_gpu_xgmi.py tests/test_gpu_syncbn.py tests/test_gpu_rccl_capture.py -x -q --timeout 300 --timeout-method thread -m gpu >> $L 2>&1 || exit 1
B="--steps 10 --warmup 3 --trials 0 --b1 0 --experiment 0 --comparator-steps 0 --full-search 0 --floor 0 --per-rank-bn 0"
for n in 2 4; do
  echo "--- $n ranks, SyncBN, small-fold path" >> $L
  timeout -k 10 400 python bench.py --gpus $n $B > gpurun_out/bn.json 2>>$L || exit 1
  python -c "import json; r=json.loads(open('gpurun_out/bn.json').read().strip().splitlines()[-1]); print(json.dumps({k: r[k] for k in ('ms_per_step','rendezvous_per_step','rendezvous_in_graph','syncbn_path','xgmi_self_test','distinct_devices')}))" >> $L || exit 1
done
echo done >> $L
