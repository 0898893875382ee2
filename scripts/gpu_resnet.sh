#!/bin/bash
# ResNet-18 trial kernels on one MI355X: BN numerics, HIP vs MIOpen batch norm throughput, kernel profile.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/resnet.log
: > $L
timeout -k 10 600 python -u -m pytest tests/test_gpu_batchnorm.py tests/test_gpu_conv.py -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit $?
for bn in hip torch; do
  echo "=== bn=$bn" >> $L
  timeout -k 10 300 python -m katib_amd.workloads.resnet_cifar --epochs 2 --max-steps 60 --bn $bn >> $L 2>&1 || exit $?
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_resnet_hip -o run -- \
  python3 -m katib_amd.workloads.resnet_cifar --epochs 1 --max-steps 40) >> $L 2>&1 || exit $?
mkdir -p $R/gpurun_out/prof_resnet_hip && find /tmp/prof_resnet_hip -name "*kernel_stats*" -exec cp {} $R/gpurun_out/prof_resnet_hip/ \;
echo done >> $L
