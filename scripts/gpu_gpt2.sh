#!/bin/bash
# GPT-2 trial kernels on one MI355X: numerics tests, flat vs module throughput, kernel profile.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/gpt2.log
: > $L
timeout -k 10 600 python -u -m pytest tests/test_gpu_transformer.py -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider >> $L 2>&1 || exit $?
for impl in flat module; do
  echo "=== $impl" >> $L
  timeout -k 10 300 python -m katib_amd.workloads.gpt2_pbt --steps ${GPT_STEPS:-30} --batch-size 16 --impl $impl >> $L 2>&1 || exit $?
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_gpt2flat -o run -- \
  python3 -m katib_amd.workloads.gpt2_pbt --steps 12 --batch-size 16 --capture 0 --impl flat) >> $L 2>&1 || exit $?
mkdir -p $R/gpurun_out/prof_gpt2flat && find /tmp/prof_gpt2flat -name "*kernel_stats*" -exec cp {} $R/gpurun_out/prof_gpt2flat/ \;
echo done >> $L
