#!/bin/bash
# whole-network Function: GPU DARTS tests, hygiene, A/B bench, timeline
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r04g.log
: > $L
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "[rc=$rc] $name $(date +%T)" >> $L
  return $rc
}
step darts-tests 600 python -u -m pytest tests/test_gpu_darts.py tests/test_gpu_graph_hygiene.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
for c in 1 0 1 0; do
  step bench-net$c 300 env KATIB_DARTS_NET_FUNCTION=$c python bench.py --steps 40 --warmup 5 --trials 0 --b1 0 --comparator-steps 0 --full-search 0 || exit 1
done
bash scripts/gpu_r04.sh tl >> $L 2>&1 || exit 1
echo done >> $L
