#!/bin/bash
# Round 5: LN backward with two rows per wave in flight - transformer numerics, GPT-2 member throughput, kernel stats.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/r05v.log
: > $L
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_transformer.py tests/test_gpt2_flat.py >> $L 2>&1 || exit 1
echo "=== gpt2 member $(date +%T)" >> $L
for rep in 1 2; do
  echo "--- ln-fused bias grads rep $rep" >> $L
  timeout -k 10 300 python -m katib_amd.workloads.gpt2_pbt --batch-size 16 --steps 40 --checkpoint-dir /tmp/g2 --save-files 0 >> $L 2>&1 || exit 1
  echo "--- colsum bias grads rep $rep" >> $L
  KATIB_GPT2_LN_BIAS=0 timeout -k 10 300 python -m katib_amd.workloads.gpt2_pbt --batch-size 16 --steps 40 --checkpoint-dir /tmp/g2 --save-files 0 >> $L 2>&1 || exit 1
done
echo "=== gpt2 prof $(date +%T)" >> $L
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_gpt2 -o run -- \
  python3 -m katib_amd.workloads.gpt2_pbt --batch-size 16 --steps 12 --checkpoint-dir /tmp/g3 --save-files 0) >> $L 2>&1 || exit 1
mkdir -p $R/gpurun_out/prof_gpt2_r05v && find /tmp/prof_gpt2 -name "*kernel_stats*" -exec cp {} $R/gpurun_out/prof_gpt2_r05v/ \;
echo done >> $L
