#!/bin/bash
# Round 5: PyTorch TunableOp selection of the hipBLASLt / rocBLAS GEMM solutions for the GPT-2 member's
# library GEMMs on MI355X - a tuning pass (eager, no graph) writes the per-shape choice, then timed runs
# with the file (tuning off) against the default heuristics.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/r05bb.log
: > $L
F=$R/gpurun_out/tunableop_gpt2_mi355x.csv
rm -f $F
echo "=== tuning $(date +%T)" >> $L
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$F \
  PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=20 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5 \
  timeout -k 10 900 python -m katib_amd.workloads.gpt2_pbt --batch-size 16 --steps 3 --capture 0 --eval-batches 1 \
  --checkpoint-dir /tmp/gt --save-files 0 >> $L 2>&1 || exit 1
ls -la $F >> $L
for rep in 1 2; do
  echo "--- default heuristics rep $rep" >> $L
  timeout -k 10 300 python -m katib_amd.workloads.gpt2_pbt --batch-size 16 --steps 40 --checkpoint-dir /tmp/g2 --save-files 0 >> $L 2>&1 || exit 1
  echo "--- tunableop file rep $rep" >> $L
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$F \
    timeout -k 10 300 python -m katib_amd.workloads.gpt2_pbt --batch-size 16 --steps 40 --checkpoint-dir /tmp/g2 --save-files 0 >> $L 2>&1 || exit 1
done
echo done >> $L
