#!/bin/bash
# PMC counters of the B5 DARTS step (eager launches): wave cycles, VALU / LDS instructions,
# LDS bank conflicts, L2 atomics per kernel. One counter pass per rocprofv3 run.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT TCC_EA0_ATOMIC_sum \
  --output-format csv -d gpurun_out/pmc_b5 -o run -- python3 bench.py --steps 2 --warmup 1 --capture 0 \
  --valid-batches 1 > gpurun_out/pmc_b5.log 2>&1 || exit $?
f=$(find gpurun_out/pmc_b5 -name '*counter_collection.csv' | head -n 1)
python3 scripts/pmc_summary.py "$f" 25 > gpurun_out/darts_b5_pmc.txt
