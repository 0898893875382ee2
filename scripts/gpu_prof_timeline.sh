#!/bin/bash
# Kernel timeline of the B5 DARTS step on one MI355X (rocprofv3 kernel trace) -> per-step span,
# kernel busy time, gaps, launches and per-family breakdown (scripts/prof_timeline.py).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${1:-b5}
rm -rf gpurun_out/prof_tl_$CFG
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_tl_$CFG -o run -- \
  python3 bench.py --config $CFG --steps 10 --warmup 3 --trials 0 --b1 0 --experiment 0 --comparator-steps 0 --full-search 0 \
  > gpurun_out/prof_tl_$CFG.log 2>&1 || exit $?
f=$(find gpurun_out/prof_tl_$CFG -name '*kernel_trace.csv' | head -n 1)
python3 scripts/prof_timeline.py "$f" virtual_step_kernel 5 > gpurun_out/darts_${CFG}_timeline.txt || exit 1
rm -rf gpurun_out/prof_tl_$CFG
