#!/bin/bash
# Round 5: fused ResNet-18 step (ops/resnet_step.py) - numerics vs fp32 autograd+SGD, the
# trial, its kernel profile; graph-captured conv kernel table vs MIOpen; DP rendezvous count on
# the default DARTS config.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/r05n.log
: > $L
echo "=== tests $(date +%T)" >> $L
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_resnet_step.py >> $L 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_workloads.py -k "resnet" >> $L 2>&1 || exit 1
echo "=== resnet run $(date +%T)" >> $L
timeout -k 10 300 python -m katib_amd.workloads.resnet_cifar --epochs 2 >> $L 2>&1 || exit 1
timeout -k 10 300 python -m katib_amd.workloads.resnet_cifar --epochs 2 --step module >> $L 2>&1 || exit 1
echo "=== resnet prof $(date +%T)" >> $L
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_resnet -o run -- \
  python3 -m katib_amd.workloads.resnet_cifar --epochs 1 --max-steps 60) >> $L 2>&1 || exit 1
mkdir -p $R/gpurun_out/prof_resnet_r05n && find /tmp/prof_resnet -name "*kernel_stats*" -exec cp {} $R/gpurun_out/prof_resnet_r05n/ \;
echo "=== conv graph table $(date +%T)" >> $L
timeout -k 10 300 python benchmarks/bench_conv.py --graph >> $L 2>&1 || exit 1
echo "=== rendezvous default $(date +%T)" >> $L
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --gpus 2 --steps 2 --warmup 1 --config default --batch 32 --trials 0 --b1 0 \
  --experiment 0 --comparator-steps 0 --full-search 0 --floor 0 >> $L 2>&1 || exit 1
echo done >> $L
echo "=== wgrad split sweep $(date +%T)" >> $L
for wg in 512 1024 2048; do for ms in 4 8 16; do
  echo "--- WG=$wg MIN_STAGES=$ms" >> $L
  KATIB_CONV_WGRAD_WG=$wg KATIB_CONV_WGRAD_MIN_STAGES=$ms timeout -k 10 120 python benchmarks/bench_conv.py --graph --hip-only >> $L 2>&1 || exit 1
done; done
echo done-sweep >> $L
