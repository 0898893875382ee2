#!/bin/bash
# conv kernels: numerics tests, per-layer bench vs MIOpen, ResNet-18 trial on both backends
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/conv.log
: > $L
timeout -k 10 600 python -m pytest tests/test_gpu_conv.py -q -x -p no:cacheprovider >> $L 2>&1 || exit 1
timeout -k 10 600 python benchmarks/bench_conv.py >> $L 2>&1 || exit 1
timeout -k 10 600 python -m katib_amd.workloads.resnet_cifar --epochs 1 --max-steps 40 >> $L 2>&1 || exit 1
echo done >> $L
