#!/bin/bash
# Round 5: ResNet-18 after set_to_none grads + num_batches_tracked folded into the BN finalize kernel:
# BN / workload GPU tests, the captured step and its kernel profile.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/r05l.log
: > $L
echo "=== tests $(date +%T)" >> $L
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_batchnorm.py tests/test_gpu_workloads.py -k "batchnorm or bn or resnet" >> $L 2>&1 || exit 1
echo "=== resnet run $(date +%T)" >> $L
timeout -k 10 300 python -m katib_amd.workloads.resnet_cifar --epochs 2 >> $L 2>&1 || exit 1
echo "=== resnet prof $(date +%T)" >> $L
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_resnet -o run -- \
  python3 -m katib_amd.workloads.resnet_cifar --epochs 1 --max-steps 60) >> $L 2>&1 || exit 1
mkdir -p $R/gpurun_out/prof_resnet_r05l && find /tmp/prof_resnet -name "*kernel_stats*" -exec cp {} $R/gpurun_out/prof_resnet_r05l/ \;
echo done >> $L
