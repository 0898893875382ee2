#!/bin/bash
# Memory-side bytes per DARTS kernel (one search step, eager): FETCH_SIZE / WRITE_SIZE in their own
# passes, with the kernel trace for durations -> achieved bandwidth per kernel.
# Usage: gpu_pmc_bw.sh [b5|default]  -> gpurun_out/darts_<config>_bw.txt
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${1:-b5}
ARGS="--steps 2 --warmup 1 --capture 0 --valid-batches 1 --trials 0 --b1 0 --experiment 0 --comparator-steps 0 --full-search 0"
[ "$CFG" = default ] && ARGS="$ARGS --config default"
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o run -- \
  python3 bench.py $ARGS > gpurun_out/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o run -- \
  python3 bench.py $ARGS > gpurun_out/pmc_write.log 2>&1 || exit $?
python3 scripts/pmc_bw.py gpurun_out/pmc_fetch gpurun_out/pmc_write > gpurun_out/darts_${CFG}_bw.txt || exit 1
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
