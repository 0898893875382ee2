#!/bin/bash
# GPU tests, then kernel profiles of the trial workloads. Stops at the first crash/timeout.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "[rc=$rc] pytest-gpu" >> gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_prof_workloads.sh
