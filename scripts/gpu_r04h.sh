#!/bin/bash
# A/B of a kernel switch: GPU DARTS tests, then bench with env VAR=0/1 alternating. Usage: gpu_r04h.sh VAR
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${1:-KATIB_HIP_POOL_BWD_SCALAR}
L=gpurun_out/r04h.log
: > $L
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "[rc=$rc] $name $(date +%T)" >> $L
  return $rc
}
step darts-tests 600 python -u -m pytest tests/test_gpu_darts.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
for c in 0 1 0 1; do
  if [ $c = 1 ]; then E="$V=1"; else E="KATIB_AB_NONE=1"; fi
  step "bench $E" 300 env $E python bench.py --steps 40 --warmup 5 --trials 0 --b1 0 --comparator-steps 0 --full-search 0 || exit 1
done
bash scripts/gpu_r04.sh tl >> $L 2>&1 || exit 1
echo done >> $L
