#!/bin/bash
# gemm256 (256x256-tile 8-wave ping-pong GEMM): numerics vs fp32, then the GPT-2 GEMM table vs hipBLASLt.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$(pwd)
L=gpurun_out/r06b.log
: > $L


echo "=== gemm256 tests $(date +%T)" >> $L
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -v --timeout 120 --timeout-method thread -m gpu -k "gemm256" >> $L 2>&1 || exit 1
timeout -k 10 200 python -u -m pytest tests/test_gpu_transformer.py -x -q --timeout 120 --timeout-method thread -m gpu -k "cross_entropy" >> $L 2>&1 || exit 1
echo "=== bench_gemm256 $(date +%T)" >> $L
timeout -k 10 400 python benchmarks/bench_gemm256.py --square --ablate >> $L 2>&1 || exit 1
echo done >> $L
echo "=== pmc $(date +%T)" >> $L
rm -rf gpurun_out/g256_pmc1 gpurun_out/g256_pmc2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/g256_pmc1 -o run -- \
  python3 scripts/gemm256_pmc_driver.py >> $L 2>&1 || exit 1
f=$(find gpurun_out/g256_pmc1 -name '*counter_collection.csv' | head -n 1)
python3 scripts/pmc_summary.py "$f" 10 >> $L 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM SQ_INSTS_LDS \
  SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/g256_pmc2 -o run -- \
  python3 scripts/gemm256_pmc_driver.py >> $L 2>&1 || exit 1
f=$(find gpurun_out/g256_pmc2 -name '*counter_collection.csv' | head -n 1)
python3 scripts/pmc_summary.py "$f" 10 >> $L 2>&1 || exit 1
rm -rf gpurun_out/g256_pmc1 gpurun_out/g256_pmc2
echo done2 >> $L
