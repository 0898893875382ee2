#!/bin/bash
# kernel profile of the DARTS default config (darts-gpu.yaml: C=16, L=3, N=4)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_darts_default
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_darts_default -o run -- \
  python3 bench.py --config default --steps 5 --warmup 2 > gpurun_out/prof_default.log 2>&1 || exit 1
f=$(find gpurun_out/prof_darts_default -name '*kernel_stats.csv' | head -n 1)
python3 scripts/prof_summary.py "$f" 40 > gpurun_out/darts_default_kernel_stats.txt || exit 1
