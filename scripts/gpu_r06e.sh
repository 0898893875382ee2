#!/bin/bash
# SyncBN rendezvous: the one-shot handshake floor per workgroup count (1 / 4 / 16) at 2 and 4 ranks sharing
# the one GPU, and the rendezvous count per B5 step with the concurrent vs stacked Hessian passes.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$(pwd)
L=gpurun_out/r06e.log
: > $L
for w in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $w --master-addr 127.0.0.1 \
    --master-port $((29700 + w)) scripts/rendezvous_probe.py >> $L 2>&1 || exit 1
done
B="--steps 10 --warmup 3 --trials 0 --b1 0 --experiment 0 --comparator-steps 0 --full-search 0 --floor 0 --per-rank-bn 0"
for h in concurrent stacked; do
  echo "--- 2 ranks, SyncBN, hessian $h" >> $L
  timeout -k 10 400 python bench.py --gpus 2 $B --hessian $h > gpurun_out/b2.json 2>>$L || exit 1
  python -c "import json; r=json.loads(open('gpurun_out/b2.json').read().strip().splitlines()[-1]); print(json.dumps({k: r[k] for k in ('ms_per_step','rendezvous_per_step','rendezvous_in_graph','syncbn_path','xgmi_self_test','distinct_devices','hessian_stack')}))" >> $L || exit 1
done
echo done >> $L
