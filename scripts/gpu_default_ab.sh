cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="--config default --steps 10 --warmup 3 --trials 0 --b1 0 --experiment 0 --comparator-steps 0 --full-search 0 --floor 0 --valid-batches 1"
for rep in 1 2; do
for lib in base new; do
  if [ $lib = base ]; then export KATIB_AMD_HIPKERN=$(pwd)/katib_amd/_hipkern_base.so; else unset KATIB_AMD_HIPKERN; fi
  timeout -k 10 300 python bench.py $B > gpurun_out/bd.json 2>/dev/null || exit 1
  echo "$lib $(python -c "import json; print(json.loads(open('gpurun_out/bd.json').read().strip().splitlines()[-1])['ms_per_step'])")"
done
done
