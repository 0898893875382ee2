#!/bin/bash
# Round 5: ResNet-18 (config 3) refresh - per-layer conv table vs MIOpen, a kernel profile of the
# training step, and the images/s of the captured step.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/r05k.log
: > $L
echo "=== conv table $(date +%T)" >> $L
timeout -k 10 300 python benchmarks/bench_conv.py >> $L 2>&1 || exit 1
echo "=== resnet run $(date +%T)" >> $L
timeout -k 10 300 python -m katib_amd.workloads.resnet_cifar --epochs 2 >> $L 2>&1 || exit 1
echo "=== resnet prof $(date +%T)" >> $L
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_resnet -o run -- \
  python3 -m katib_amd.workloads.resnet_cifar --epochs 1 --max-steps 60) >> $L 2>&1 || exit 1
mkdir -p $R/gpurun_out/prof_resnet_r05 && find /tmp/prof_resnet -name "*kernel_stats*" -exec cp {} $R/gpurun_out/prof_resnet_r05/ \;
echo done >> $L
