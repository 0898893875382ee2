#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
L=gpurun_out/r05h.log
: > $L
for o in adam sgd ftrl; do
  echo "=== $o" >> $L
  timeout -k 10 120 python scripts/trial_model_phase_probe.py $o >> $L 2>&1 || exit 1
done
