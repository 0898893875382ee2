#!/bin/bash
# Kernel profile of the headline DARTS bench (B5 and darts-gpu.yaml default configs).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in b5 default; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_darts_$cfg -o run -- \
    python3 bench.py --config $cfg --steps 10 --warmup 3 > gpurun_out/prof_darts_$cfg.log 2>&1 || exit $?
  f=$(find gpurun_out/prof_darts_$cfg -name '*kernel_stats.csv' | head -n 1)
  python3 scripts/prof_summary.py "$f" 40 > gpurun_out/darts_${cfg}_kernel_stats.txt || exit 1
done
