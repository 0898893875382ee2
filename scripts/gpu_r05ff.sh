#!/bin/bash
# Round 5: rotated-component LDS scatter in the DARTS plane kernels' staging (lds_put4) - DARTS GPU
# tests, then B5 and darts-gpu.yaml step time A/B against the in-order build (KATIB_DARTS_LDS_ROTATE=0),
# then the LDS counters of the B5 step.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/r05ff.log
: > $L
NOROT=$R/katib_amd/_hipkern_norot$(python -c "import sysconfig; print(sysconfig.get_config_var('EXT_SUFFIX'))")
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_darts.py tests/test_gpu_darts_bf16.py tests/test_gpu_dwconv.py >> $L 2>&1 || exit 1
B="--trials 0 --b1 0 --experiment 0 --comparator-steps 0 --full-search 0"
for rep in 1 2 3; do
  echo "--- rotate b5 rep $rep" >> $L
  timeout -k 10 300 python bench.py --steps 60 --warmup 5 $B >> $L 2>&1 || exit 1
  echo "--- in-order b5 rep $rep" >> $L
  KATIB_AMD_HIPKERN=$NOROT timeout -k 10 300 python bench.py --steps 60 --warmup 5 $B >> $L 2>&1 || exit 1
done
for rep in 1 2; do
  echo "--- rotate default rep $rep" >> $L
  timeout -k 10 300 python bench.py --config default --steps 20 --warmup 3 $B >> $L 2>&1 || exit 1
  echo "--- in-order default rep $rep" >> $L
  KATIB_AMD_HIPKERN=$NOROT timeout -k 10 300 python bench.py --config default --steps 20 --warmup 3 $B >> $L 2>&1 || exit 1
done
echo done >> $L
