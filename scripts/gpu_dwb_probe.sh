#!/bin/bash
# dw_bwd_plane phase costs: kernel stats with input grads (1) / weight grads (2) skipped
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for d in 0 1 2 3; do
  rm -rf gpurun_out/prof_dwb_$d
  KATIB_HIP_DWB_DBG=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dwb_$d -o run -- \
    python3 bench.py --steps 10 --warmup 3 > gpurun_out/dwb_$d.log 2>&1 || exit 1
  f=$(find gpurun_out/prof_dwb_$d -name '*kernel_stats.csv' | head -n 1)
  python3 scripts/prof_summary.py "$f" 60 > gpurun_out/dwb_stats_$d.txt || exit 1
done
