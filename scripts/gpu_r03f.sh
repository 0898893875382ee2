#!/bin/bash
# N>1 rehearsal of the driver's bench on a one-GPU box: bench.py under torch.distributed.run with
# 2 ranks sharing device 0 (gloo control plane + the one-shot IPC all-reduce inside the graph),
# strong and weak scaling; then the darts-gpu.yaml default config at N=1.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r03f.log
: > $L
for sc in strong weak; do
  echo "=== dp2 shared-device $sc" >> $L
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29611 bench.py --gpus 2 --steps 20 --warmup 5 --trials 0 --comparator-steps 0 \
    --full-search 0 --scaling $sc >> $L 2>&1 || exit 1
done
echo "=== default n1" >> $L
timeout -k 10 400 python bench.py --config default --steps 10 --warmup 3 --trials 0 --comparator-steps 0 \
  --full-search 0 >> $L 2>&1 || exit 1
echo done >> $L
