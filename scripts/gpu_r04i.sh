#!/bin/bash
# A/B of the plane kernels' 4-pixel output paths (KATIB_HIP_VEC_MASK 0 / 5 / 15) on the B5 step and
# the darts-gpu.yaml step, after the GPU DARTS tests with every path on (mask 15) and the default.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r04i.log
: > $L
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "[rc=$rc] $name $(date +%T)" >> $L
  return $rc
}
T="python -u -m pytest tests/test_gpu_darts.py tests/test_gpu_darts_default.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
[ -f tests/test_gpu_darts_default.py ] || T="python -u -m pytest tests/test_gpu_darts.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
step "darts-tests mask15" 600 env KATIB_HIP_VEC_MASK=15 $T || exit 1
step "darts-tests default" 600 $T || exit 1
Q="--trials 0 --b1 0 --comparator-steps 0 --full-search 0"
for r in 1 2; do
  for m in 0 5 15; do
    step "b5 mask$m" 300 env KATIB_HIP_VEC_MASK=$m python bench.py --steps 40 --warmup 5 $Q || exit 1
  done
done
for m in 0 5 15; do
  step "default mask$m" 300 env KATIB_HIP_VEC_MASK=$m python bench.py --config default --steps 10 --warmup 3 $Q || exit 1
done
echo done >> $L
