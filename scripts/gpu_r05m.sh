#!/bin/bash
# Round 5: graph-captured kernel-level conv table (HIP implicit GEMM vs MIOpen), ResNet-18 shapes.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$(pwd)
L=gpurun_out/r05m.log
: > $L
timeout -k 10 300 python benchmarks/bench_conv.py --graph >> $L 2>&1 || exit 1
echo done >> $L
# rendezvous per step of the HIP DP step on the default config (2 ranks sharing the one GPU)
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --gpus 2 --steps 2 --warmup 1 --config default --batch 32 --trials 0 --b1 0 \
  --experiment 0 --comparator-steps 0 --full-search 0 --floor 0 >> $L 2>&1 || exit 1
echo done2 >> $L
