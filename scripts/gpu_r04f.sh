#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r04f.log
: > $L
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "[rc=$rc] $name $(date +%T)" >> $L
  return $rc
}
for d in fp32 bf16 fp32 bf16; do
  step bench-$d 300 python bench.py --dtype $d --steps 40 --warmup 5 --trials 0 --b1 0 --comparator-steps 0 --full-search 0 || exit 1
done
step pmc-sq 400 bash scripts/gpu_pmc_sq.sh || exit 1
echo done >> $L
