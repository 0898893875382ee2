#!/bin/bash
# Round 5: fc1 bias-gradient column sums from the fc2 dgrad epilogue (gemm_lt colpart + reduce_rows) vs a colsum
# pass over du (KATIB_GELU_DGRAD_BIAS=0): numerics, GPT-2 member tokens/s A/B, kernel table.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/r05ii.log
: > $L
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_transformer.py tests/test_gpt2_flat.py >> $L 2>&1 || exit 1
for rep in 1 2 3; do
  echo "--- epilogue bias sums rep $rep" >> $L
  timeout -k 10 300 python -m katib_amd.workloads.gpt2_pbt --batch-size 16 --steps 40 --checkpoint-dir /tmp/g2 --save-files 0 >> $L 2>&1 || exit 1
  echo "--- colsum pass rep $rep" >> $L
  KATIB_GELU_DGRAD_BIAS=0 timeout -k 10 300 python -m katib_amd.workloads.gpt2_pbt --batch-size 16 --steps 40 --checkpoint-dir /tmp/g2 --save-files 0 >> $L 2>&1 || exit 1
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_gb -o run -- python3 -m katib_amd.workloads.gpt2_pbt --batch-size 16 --steps 20 --checkpoint-dir /tmp/g3 --save-files 0 >> $R/$L 2>&1 || exit 1
echo done >> $R/$L
