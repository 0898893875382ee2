#!/bin/bash
# Round 5: LDS-patch 3x3 / s1 conv kernel (fwd + dgrad): numerics, graph-captured conv table (on / off), ResNet step tests.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/r05x.log
: > $L
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_conv.py >> $L 2>&1 || exit 1
echo "=== conv table patch on $(date +%T)" >> $L
timeout -k 10 300 python benchmarks/bench_conv.py --graph >> $L 2>&1 || exit 1
echo "=== conv table patch 16/32-wide only $(date +%T)" >> $L
KATIB_CONV_PATCH=1 timeout -k 10 120 python benchmarks/bench_conv.py --graph --hip-only >> $L 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_resnet_step.py tests/test_gpu_workloads.py -k "resnet" >> $L 2>&1 || exit 1
echo "=== resnet run $(date +%T)" >> $L
timeout -k 10 300 python -m katib_amd.workloads.resnet_cifar --epochs 2 >> $L 2>&1 || exit 1
echo done >> $L
