#!/bin/bash
# bf16-intermediates DARTS variant: numerics (fp32 build + bf16 build vs the torch oracle), then
# fp32 vs bf16 bench on B5 and the darts-gpu.yaml default config.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r03d.log
: > $L
echo "=== tests" >> $L
timeout -k 10 900 python -u -m pytest tests/test_gpu_darts_bf16.py tests/test_gpu_darts.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit 1
for dt in fp32 bf16 fp32 bf16; do
  echo "=== $dt b5" >> $L
  timeout -k 10 300 python bench.py --dtype $dt --steps 30 --warmup 5 --trials 0 --comparator-steps 0 --full-search 0 >> $L 2>&1 || exit 1
done
for dt in fp32 bf16; do
  echo "=== $dt default" >> $L
  timeout -k 10 300 python bench.py --dtype $dt --config default --steps 10 --warmup 3 --trials 0 --comparator-steps 0 --full-search 0 >> $L 2>&1 || exit 1
done
echo done >> $L
