#!/bin/bash
# kernel profile of the DARTS B5 config (C=4, L=2, N=3) on one MI355X
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_darts_b5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_darts_b5 -o run -- \
  python3 bench.py --steps 10 --warmup 3 --full-search 0 > gpurun_out/prof_b5.log 2>&1 || exit 1
f=$(find gpurun_out/prof_darts_b5 -name '*kernel_stats.csv' | head -n 1)
python3 scripts/prof_summary.py "$f" 45 > gpurun_out/darts_b5_kernel_stats.txt || exit 1
python3 scripts/prof_families.py "$f" 25 > gpurun_out/darts_b5_families.txt || exit 1
