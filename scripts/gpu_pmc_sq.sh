#!/bin/bash
# SQ counters per DARTS kernel (one search step, eager): waves, wave-cycles, busy, wait, instruction
# mix; a second pass for VALU / LDS activity and LDS bank conflicts.
# Usage: gpu_pmc_sq.sh [b5|default] -> gpurun_out/darts_<config>_pmc_sq.txt, ..._pmc_lds.txt
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${1:-b5}
ARGS="--steps 2 --warmup 1 --capture 0 --valid-batches 1 --trials 0 --b1 0 --experiment 0 --comparator-steps 0 --full-search 0"
[ "$CFG" = default ] && ARGS="$ARGS --config default"
rm -rf gpurun_out/pmc_sq gpurun_out/pmc_lds
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU \
  SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_sq -o run -- \
  python3 bench.py $ARGS > gpurun_out/pmc_sq.log 2>&1 || exit $?
f=$(find gpurun_out/pmc_sq -name '*counter_collection.csv' | head -n 1)
python3 scripts/pmc_summary.py "$f" 25 > gpurun_out/darts_${CFG}_pmc_sq.txt || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM \
  SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_lds -o run -- \
  python3 bench.py $ARGS > gpurun_out/pmc_lds.log 2>&1 || exit $?
f=$(find gpurun_out/pmc_lds -name '*counter_collection.csv' | head -n 1)
python3 scripts/pmc_summary.py "$f" 25 > gpurun_out/darts_${CFG}_pmc_lds.txt || exit 1
rm -rf gpurun_out/pmc_sq gpurun_out/pmc_lds
