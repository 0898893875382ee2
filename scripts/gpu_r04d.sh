#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r04d.log
: > $L
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "[rc=$rc] $name $(date +%T)" >> $L
  return $rc
}
step new-tests 700 python -u -m pytest tests/test_gpu_syncbn.py tests/test_gpu_graph_hygiene.py -v -s --timeout 500 --timeout-method thread -p no:cacheprovider
step pmc-bw 600 bash scripts/gpu_pmc_bw.sh || exit 1
step bench-dp2 400 python bench.py --gpus 2 --steps 20 --warmup 5 --trials 0 --b1 0 --comparator-steps 0 --full-search 0 || exit 1
step bench-dp2-perrank 400 python bench.py --gpus 2 --steps 20 --warmup 5 --trials 0 --b1 0 --comparator-steps 0 --full-search 0 --sync-bn 0 --floor 0 || exit 1
for b in 64 32 16; do
  step bench-b$b 300 python bench.py --batch $b --steps 20 --warmup 5 --trials 0 --b1 0 --comparator-steps 0 --full-search 0 || exit 1
done
step bench-full 900 python bench.py || exit 1
echo done >> $L
