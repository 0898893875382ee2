#!/bin/bash
# Round 5: DP projection inputs - per-rank floors (B5 / default at per-rank batch 128/64/32/16, dp1),
# the rendezvous count of a SyncBN step (2 ranks sharing the GPU), the one-shot rendezvous floor
# (2 and 4 ranks, same GPU); and PBT GPT-2 at 32 trials (exploit hand-offs).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
L=gpurun_out/r05j.log
: > $L
Q="--trials 0 --b1 0 --comparator-steps 0 --full-search 0"
for b in 128 64 32 16; do
  echo "=== b5 batch $b $(date +%T)" >> $L
  timeout -k 10 300 python bench.py --steps 40 --warmup 5 --batch $b $Q >> $L 2>&1 || exit 1
done
for b in 128 64 32 16; do
  echo "=== default batch $b $(date +%T)" >> $L
  timeout -k 10 300 python bench.py --config default --steps 10 --warmup 3 --batch $b $Q >> $L 2>&1 || exit 1
done
echo "=== 2-rank syncbn shared GPU $(date +%T)" >> $L
timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 --floor 0 $Q >> $L 2>&1 || exit 1
for w in 2 4; do
  echo "=== rendezvous probe world $w $(date +%T)" >> $L
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $w --master-addr 127.0.0.1 \
    --master-port $((29600 + w)) scripts/rendezvous_probe.py >> $L 2>&1 || exit 1
done
echo "=== pbt 32 $(date +%T)" >> $L
timeout -k 10 600 python scripts/experiments_r05.py --only pbt-gpt2 --pbt-trials 32 >> $L 2>&1 || exit 1
echo done >> $L
