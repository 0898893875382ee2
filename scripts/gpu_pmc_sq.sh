#!/bin/bash
# SQ counters per DARTS kernel (B5 step, eager): waves, wave-cycles, busy, wait, instruction mix.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_sq
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU \
  SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_sq -o run -- \
  python3 bench.py --steps 2 --warmup 1 --capture 0 --valid-batches 1 --trials 0 --b1 0 --comparator-steps 0 --full-search 0 > gpurun_out/pmc_sq.log 2>&1 || exit $?
f=$(find gpurun_out/pmc_sq -name '*counter_collection.csv' | head -n 1)
python3 scripts/pmc_summary.py "$f" 25 > gpurun_out/darts_b5_pmc_sq.txt
