#!/bin/bash
# Fused MLP kernels on one MI355X: numerics, HIP vs module trial time, trials/hour bench, profile.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/mlp.log
: > $L
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider >> $L 2>&1 || exit $?
for impl in hip module; do
  echo "=== impl=$impl" >> $L
  timeout -k 10 300 python -m katib_amd.workloads.mnist_mlp --epochs 3 --impl $impl >> $L 2>&1 || exit $?
done
echo "=== bench-trials" >> $L
timeout -k 10 600 python bench_trials.py --trials 24 --parallel 8 --epochs 3 >> $L 2>&1 || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_mlp_hip -o run -- \
  python3 -m katib_amd.workloads.mnist_mlp --epochs 3) >> $L 2>&1 || exit $?
mkdir -p $R/gpurun_out/prof_mlp_hip && find /tmp/prof_mlp_hip -name "*kernel_stats*" -exec cp {} $R/gpurun_out/prof_mlp_hip/ \;
echo done >> $L
