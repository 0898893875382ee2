#!/bin/bash
# Round 5: GPT-2 PBT member with the layout-native backward GEMMs: transformer GPU tests, member
# throughput A/B (KATIB_HIP_GEMM_BWD=0 hipBLASLt vs auto), kernel profile of the new default.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/r05f.log
: > $L
timeout -k 10 400 python -u -m pytest tests/test_gpu_transformer.py tests/test_gpu_gemm.py -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit 1
for r in 1 2; do
  for m in 0 auto; do
    echo "=== KATIB_HIP_GEMM_BWD=$m" >> $L
    timeout -k 10 300 env KATIB_HIP_GEMM_BWD=$m python -m katib_amd.workloads.gpt2_pbt --steps 30 --batch-size 16 --impl flat >> $L 2>&1 || exit 1
  done
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_gpt2 -o run -- \
  python3 -m katib_amd.workloads.gpt2_pbt --steps 12 --batch-size 16 --capture 0 --impl flat) >> $L 2>&1 || exit 1
mkdir -p $R/gpurun_out/prof_gpt2_r05 && find /tmp/prof_gpt2 -name "*kernel_stats*" -exec cp {} $R/gpurun_out/prof_gpt2_r05/ \;
echo done >> $L
