#!/bin/bash
# Round 5: phase-split strided dgrad + new wgrad split policy: conv numerics, fused ResNet step,
# graph-captured conv table vs MIOpen, the trial, its profile.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/r05p.log
: > $L
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_conv.py tests/test_gpu_resnet_step.py >> $L 2>&1 || exit 1
echo "=== conv graph table $(date +%T)" >> $L
timeout -k 10 300 python benchmarks/bench_conv.py --graph >> $L 2>&1 || exit 1
echo "=== phases off $(date +%T)" >> $L
KATIB_CONV_DGRAD_PHASES=0 timeout -k 10 120 python benchmarks/bench_conv.py --graph --hip-only >> $L 2>&1 || exit 1
echo "=== resnet run $(date +%T)" >> $L
timeout -k 10 300 python -m katib_amd.workloads.resnet_cifar --epochs 2 >> $L 2>&1 || exit 1
echo done >> $L
