#!/bin/bash
# bf16 GEMM pipeline-depth sweep: numerics + GPT-2 forward projection bench per KATIB_HIP_GEMM_STAGES
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
L=gpurun_out/gemm_stages.log
: > $L
for s in ${@:-3 4 2}; do
  echo "=== STAGES=$s" >> $L
  KATIB_HIP_GEMM_STAGES=$s timeout -k 10 200 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit 1
  KATIB_HIP_GEMM_STAGES=$s timeout -k 10 200 python benchmarks/bench_gemm.py >> $L 2>&1 || exit 1
done
echo done >> $L
