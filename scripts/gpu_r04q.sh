#!/bin/bash
# Round-4 refresh of the non-DARTS workloads on one MI355X: GPT-2 PBT member, ResNet-18 (HyperBand
# trial), MNIST MLP (TPE trial), ENAS controller GetSuggestions, each under its own limit.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r04q.log
: > $L
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)" >> $L
  local s=$(date +%s.%N)
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "[rc=$rc] $name $(date +%T) wall_s=$(echo "$(date +%s.%N) - $s" | bc)" >> $L
  return $rc
}
step gpt2-flat 300 python -m katib_amd.workloads.gpt2_pbt --steps 30 --batch-size 16 --impl flat || exit 1
step resnet 300 python -m katib_amd.workloads.resnet_cifar --epochs 1 --max-steps 60 || exit 1
step mlp 300 python -m katib_amd.workloads.mnist_mlp --epochs 3 || exit 1
step enas-ctrl 300 python benchmarks/bench_enas_ctrl.py || exit 1
echo done >> $L
