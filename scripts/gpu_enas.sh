#!/bin/bash
# ENAS controller kernel on one MI355X: numerics vs the torch oracle, GetSuggestions cost, kernel profile.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/enas.log
: > $L
timeout -k 10 600 python -u -m pytest tests/test_gpu_enas.py tests/test_gpu_darts.py -k "enas or Enas or combine" -x -v \
  --timeout 120 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit $?
timeout -k 10 300 python benchmarks/bench_enas_ctrl.py >> $L 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_enas -o run -- \
  python3 benchmarks/bench_enas_ctrl.py --backends hip --reps 3 >> $L 2>&1 || exit $?
f=$(find gpurun_out/prof_enas -name '*kernel_stats.csv' | head -n 1)
python3 scripts/prof_summary.py "$f" 20 > gpurun_out/enas_kernel_stats.txt || exit 1
echo done >> $L
