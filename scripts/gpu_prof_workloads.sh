#!/bin/bash
# Kernel profiles of the trial workloads (GPT-2 small PBT member, ResNet-18, MNIST MLP).
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$R
L=gpurun_out/prof_wl.log
: > $L
prof() {  # prof <name> <args...>
  local name=$1; shift
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$name -o run -- python3 "$@") >> $L 2>&1
  local rc=$?
  echo "[rc=$rc] $name" >> $L
  mkdir -p $R/gpurun_out/prof_$name && find /tmp/prof_$name -name "*kernel_stats*" -exec cp {} $R/gpurun_out/prof_$name/ \;
  return $rc
}
prof gpt2 -m katib_amd.workloads.gpt2_pbt --steps ${GPT_STEPS:-12} --batch-size 16 --capture 0 || exit 1
prof resnet -m katib_amd.workloads.resnet_cifar --epochs 1 --max-steps 40 || exit 1
prof mlp -m katib_amd.workloads.mnist_mlp --epochs 3 || exit 1
echo done >> $L
