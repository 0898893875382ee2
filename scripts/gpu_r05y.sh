#!/bin/bash
# Round 5: ResNet-18 fused step with the patch conv kernels + parallel head reduction: tests, trial, kernel profile.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/r05y.log
: > $L
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_resnet_step.py tests/test_gpu_conv.py >> $L 2>&1 || exit 1
echo "=== resnet run $(date +%T)" >> $L
timeout -k 10 300 python -m katib_amd.workloads.resnet_cifar --epochs 2 >> $L 2>&1 || exit 1
echo "=== resnet prof $(date +%T)" >> $L
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_resnet -o run -- \
  python3 -m katib_amd.workloads.resnet_cifar --epochs 1 --max-steps 60) >> $L 2>&1 || exit 1
mkdir -p $R/gpurun_out/prof_resnet_r05y && find /tmp/prof_resnet -name "*kernel_stats*" -exec cp {} $R/gpurun_out/prof_resnet_r05y/ \;
echo done >> $L
