#!/bin/bash
# Round 5 final DARTS tables (current kernels): timeline, per-kernel bandwidth, SQ / LDS counters for
# B5 and darts-gpu.yaml. Each rocprofv3 pass in its own run (no --pmc with trace domains).
set -o pipefail
cd "$(dirname "$0")/.."
for cfg in b5 default; do
  bash scripts/gpu_prof_timeline.sh $cfg || exit 1
  bash scripts/gpu_pmc_bw.sh $cfg || exit 1
  bash scripts/gpu_pmc_sq.sh $cfg || exit 1
done
echo done > gpurun_out/r05u.done
