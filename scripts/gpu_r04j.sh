#!/bin/bash
# pw_bwd_wave per-workgroup channel groups, LDS-staged 4-pixel pool forward (A/B KATIB_HIP_POOL_FWD_SCALAR),
# stride-2 parity classes in dw_bwd_plane (mask bit 4), band knob KATIB_HIP_DWB_MIN_WG,
# pools in the stage-1 dw-pw launch (A/B KATIB_HIP_JOINT_POOL=0), narrow pw_fwd_px (A/B KATIB_HIP_PW_FWD_TILED=1): GPU DARTS tests, B5 + default-config benches (vector-path
# masks 5 / 13 on the default config), the default-config timeline and SQ / LDS / MFMA counters.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r04j.log
: > $L
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "[rc=$rc] $name $(date +%T)" >> $L
  return $rc
}
step darts-tests-joint-off 600 env KATIB_HIP_JOINT_POOL=0 python -u -m pytest tests/test_gpu_darts.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step darts-tests 600 python -u -m pytest tests/test_gpu_darts.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step darts-tests-mask0 600 env KATIB_HIP_VEC_MASK=0 KATIB_HIP_PW_FWD_TILED=1 python -u -m pytest tests/test_gpu_darts.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
Q="--trials 0 --b1 0 --comparator-steps 0 --full-search 0"
for r in 1 2; do
  step "b5" 300 python bench.py --steps 40 --warmup 5 $Q || exit 1
  step "b5 joint-pool-off" 300 env KATIB_HIP_JOINT_POOL=0 python bench.py --steps 40 --warmup 5 $Q || exit 1
  step "b5 pw-fwd-tiled" 300 env KATIB_HIP_PW_FWD_TILED=1 python bench.py --steps 40 --warmup 5 $Q || exit 1
  step "b5 s2-class-off (mask5)" 300 env KATIB_HIP_VEC_MASK=5 python bench.py --steps 40 --warmup 5 $Q || exit 1
  step "b5 dwb-min-wg4096" 300 env KATIB_HIP_DWB_MIN_WG=4096 python bench.py --steps 40 --warmup 5 $Q || exit 1
  step "b5 joint-off pool-fwd-scalar" 300 env KATIB_HIP_JOINT_POOL=0 KATIB_HIP_POOL_FWD_SCALAR=1 python bench.py --steps 40 --warmup 5 $Q || exit 1
done
for m in 21 5 29; do
  step "default mask$m" 300 env KATIB_HIP_VEC_MASK=$m python bench.py --config default --steps 10 --warmup 3 $Q || exit 1
done
step "default pool-fwd-scalar" 300 env KATIB_HIP_POOL_FWD_SCALAR=1 python bench.py --config default --steps 10 --warmup 3 $Q || exit 1
bash scripts/gpu_r04.sh dtl >> $L 2>&1 || exit 1
bash scripts/gpu_pmc_sq.sh default >> $L 2>&1 || exit 1
echo done >> $L
