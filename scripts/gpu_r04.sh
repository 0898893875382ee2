#!/bin/bash
# Round-4 GPU steps on one MI355X. Usage: scripts/gpu_r04.sh <step>...
#   tests    pytest -m gpu + smoke
#   bench    default bench.py (B5, trials/h, comparators)
#   quick    B5 step only (no trials/h, no comparators)
#   tl       rocprofv3 kernel timeline of the B5 step -> gpurun_out/darts_b5_timeline.txt
#   default  darts-gpu.yaml config
#   dtl      rocprofv3 kernel timeline of the darts-gpu.yaml step -> gpurun_out/darts_default_timeline.txt
#   gemm     GPT-2 GEMM per-shape table, forward + dgrad + wgrad vs hipBLASLt
#   gpt2     GPT-2 PBT flat step throughput + rocprofv3 kernel stats -> gpurun_out/gpt2_kernel_stats_r04.csv
#   gbar     grid-barrier vs kernel-boundary probe (scripts/grid_barrier_probe, built on the CPU side)
# Each GPU step has its own limit; stop at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r04.log
: > $L
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "[rc=$rc] $name $(date +%T)" >> $L
  return $rc
}
for s in "$@"; do
  case $s in
    tests)
      step pytest-gpu 1200 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider || exit 1
      step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    bench) step bench 600 python bench.py || exit 1 ;;
    quick) step quick 300 python bench.py --trials 0 --b1 0 --comparator-steps 0 --full-search 0 || exit 1 ;;
    default) step default 400 python bench.py --config default --steps 10 --warmup 3 --trials 0 --b1 0 --comparator-steps 0 --full-search 0 || exit 1 ;;
    tl)
      rm -rf gpurun_out/prof_tl
      step tl 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_tl -o run -- \
        python3 bench.py --steps 10 --warmup 3 --trials 0 --b1 0 --comparator-steps 0 --full-search 0 || exit 1
      f=$(find gpurun_out/prof_tl -name '*kernel_trace.csv' | head -n 1)
      python3 scripts/prof_timeline.py "$f" virtual_step_kernel 5 > gpurun_out/darts_b5_timeline.txt || exit 1
      python3 scripts/prof_sequence.py "$f" virtual_step_kernel > gpurun_out/darts_b5_sequence.txt 2>&1 || true
      rm -rf gpurun_out/prof_tl ;;
    dtl)
      rm -rf gpurun_out/prof_dtl
      step dtl 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_dtl -o run -- \
        python3 bench.py --config default --steps 8 --warmup 3 --trials 0 --b1 0 --comparator-steps 0 --full-search 0 || exit 1
      f=$(find gpurun_out/prof_dtl -name '*kernel_trace.csv' | head -n 1)
      python3 scripts/prof_timeline.py "$f" virtual_step_kernel 5 > gpurun_out/darts_default_timeline.txt || exit 1
      rm -rf gpurun_out/prof_dtl ;;
    gbar)
      step gbar-200 120 scripts/grid_barrier_probe 200 || exit 1
      step gbar-50 120 scripts/grid_barrier_probe 50 || exit 1 ;;
    gemm) step gemm 400 python benchmarks/bench_gemm.py --backward || exit 1 ;;
    gpt2)
      step gpt2-flat 300 python -m katib_amd.workloads.gpt2_pbt --steps 30 --batch-size 16 --impl flat || exit 1
      rm -rf gpurun_out/prof_gpt2
      step gpt2-prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gpt2 -o run -- \
        python3 -m katib_amd.workloads.gpt2_pbt --steps 12 --batch-size 16 --impl flat || exit 1
      f=$(find gpurun_out/prof_gpt2 -name '*kernel_stats.csv' | head -n 1)
      cp "$f" gpurun_out/gpt2_kernel_stats_r04.csv
      rm -rf gpurun_out/prof_gpt2 ;;
    *) echo "unknown step $s" >> $L; exit 2 ;;
  esac
done
echo done >> $L
