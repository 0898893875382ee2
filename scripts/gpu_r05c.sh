#!/bin/bash
# Round 5: phase stamps of the DARTS plane kernels (diagnostic build) on B5 and darts-gpu.yaml.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r05c.log
: > $L
timeout -k 10 300 python scripts/darts_phase_stamps.py --calls 8 >> $L 2>&1 || exit 1
echo "=== default" >> $L
timeout -k 10 300 python scripts/darts_phase_stamps.py --config default --calls 4 >> $L 2>&1 || exit 1
echo done >> $L
