#!/bin/bash
# Round 5: GPT-2 member throughput + kernel table after the attention rewrite; DARTS kernels with
# VGPR-form MFMA accumulators (variant build _hipkern_vgpr) A/B on B5 and darts-gpu.yaml + numerics.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/r05t.log
: > $L
V=$R/katib_amd/_hipkern_vgpr.cpython-310-x86_64-linux-gnu.so
echo "=== gpt2 member $(date +%T)" >> $L
for rep in 1 2; do
  timeout -k 10 300 python -m katib_amd.workloads.gpt2_pbt --batch-size 16 --steps 40 --checkpoint-dir /tmp/g2 --save-files 0 >> $L 2>&1 || exit 1
done
echo "=== gpt2 prof $(date +%T)" >> $L
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_gpt2 -o run -- \
  python3 -m katib_amd.workloads.gpt2_pbt --batch-size 16 --steps 12 --checkpoint-dir /tmp/g3 --save-files 0) >> $L 2>&1 || exit 1
mkdir -p $R/gpurun_out/prof_gpt2_r05t && find /tmp/prof_gpt2 -name "*kernel_stats*" -exec cp {} $R/gpurun_out/prof_gpt2_r05t/ \;
echo "=== darts vgpr numerics $(date +%T)" >> $L
KATIB_AMD_HIPKERN=$V timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_darts.py tests/test_darts_parity.py >> $L 2>&1 || exit 1
B5="--steps 40 --warmup 5 --trials 0 --b1 0 --experiment 0 --comparator-steps 0 --full-search 0"
DF="--config default --steps 10 --warmup 3 --trials 0 --b1 0 --experiment 0 --comparator-steps 0 --full-search 0"
for rep in 1 2; do
  echo "--- b5 default-build rep $rep" >> $L
  timeout -k 10 300 python bench.py $B5 >> $L 2>&1 || exit 1
  echo "--- b5 vgpr-build rep $rep" >> $L
  KATIB_AMD_HIPKERN=$V timeout -k 10 300 python bench.py $B5 >> $L 2>&1 || exit 1
  echo "--- default-config default-build rep $rep" >> $L
  timeout -k 10 300 python bench.py $DF >> $L 2>&1 || exit 1
  echo "--- default-config vgpr-build rep $rep" >> $L
  KATIB_AMD_HIPKERN=$V timeout -k 10 300 python bench.py $DF >> $L 2>&1 || exit 1
done
echo done >> $L
