set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/fold_exp.log
: > $L
timeout -k 10 600 python -u -m pytest tests/test_gpu_darts.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit $?
KATIB_HIP_FOLD=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_darts.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit $?
for f in 1 0 1 0; do KATIB_HIP_FOLD=$f timeout -k 10 300 python bench.py --steps 30 --warmup 5 | sed "s/^/FOLD=$f /" >> $L 2>&1 || exit $?; done
echo done >> $L
