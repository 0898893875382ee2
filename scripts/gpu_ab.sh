#!/bin/bash
# Generic DARTS A/B on one MI355X: numerics tests, then B5 (and default) bench with ENV=a vs ENV=b,
# then the B5 kernel timeline of the default setting.
#   bash scripts/gpu_ab.sh <ENVVAR> <value_a> <value_b> [tests-selector]
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$1; A=$2; B=$3; SEL=${4:-tests/test_gpu_darts.py}
L=gpurun_out/ab_${V}.log
: > $L
echo "=== tests $SEL" >> $L
timeout -k 10 900 python -u -m pytest $SEL -x -q --timeout 300 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit 1
for m in $A $B $A $B; do
  echo "=== $V=$m b5" >> $L
  env $V=$m timeout -k 10 300 python bench.py --steps 30 --warmup 5 --trials 0 --comparator-steps 0 --full-search 0 >> $L 2>&1 || exit 1
done
for m in $A $B; do
  echo "=== $V=$m default" >> $L
  env $V=$m timeout -k 10 300 python bench.py --config default --steps 10 --warmup 3 --trials 0 --comparator-steps 0 --full-search 0 >> $L 2>&1 || exit 1
done
bash scripts/gpu_prof_timeline.sh b5 || exit 1
echo done >> $L
