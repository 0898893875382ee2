#!/bin/bash
# Round 5: hipBLASLt epilogue GEMMs for the GPT-2 MLP (GELU_AUX_BIAS forward, DGELU_BGRAD backward) -
# numerics, then GPT-2 member tokens/s A/B against the separate gelu / colsum kernels, then a kernel table.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/r05dd.log
: > $L
timeout -k 10 100 python scripts/lt_probe.py > gpurun_out/lt_probe.log 2>&1 && timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_transformer.py tests/test_gpt2_flat.py >> $L 2>&1 || exit 1
for rep in 1 2 3; do
  echo "--- lt bgradb rep $rep" >> $L
  timeout -k 10 300 python -m katib_amd.workloads.gpt2_pbt --batch-size 16 --steps 40 --checkpoint-dir /tmp/g2 --save-files 0 >> $L 2>&1 || exit 1
  echo "--- wgrad + colsum rep $rep" >> $L
  KATIB_LT_EPILOGUE=0 timeout -k 10 300 python -m katib_amd.workloads.gpt2_pbt --batch-size 16 --steps 40 --checkpoint-dir /tmp/g2 --save-files 0 >> $L 2>&1 || exit 1
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_lt -o run -- python3 -m katib_amd.workloads.gpt2_pbt --batch-size 16 --steps 20 --checkpoint-dir /tmp/g3 --save-files 0 >> $R/$L 2>&1 || exit 1
echo done >> $R/$L
