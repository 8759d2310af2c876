# Step leg of bench.py at several batch sizes for the shipped library and each variant given,
# interleaved over ROUNDS rounds (same box). Usage: ROUNDS=2 SIZES="1048576 8388608" bash tools/gpu_ab_size.sh tools/variants/lib_x.so ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abs
ROUNDS=${ROUNDS:-2}
SIZES=${SIZES:-"1048576 8388608"}
for r in $(seq 1 "$ROUNDS"); do
  for e in $SIZES; do
    for lib in default "$@"; do
      tag=$(basename "$lib" .so)
      if [ "$lib" = default ]; then unset MERGING_HIP_LIB; else export MERGING_HIP_LIB=$PWD/$lib; fi
      timeout -k 10 200 python bench.py --envs $e --steps 300 --no-cpu-baseline --rollout-steps 0 --qnet-launches 0 \
        --replay-stores 0 --size2-envs 0 > gpurun_out/abs/${tag}_${e}_r$r.log 2>&1 || { echo "$tag $e failed"; tail -3 gpurun_out/abs/${tag}_${e}_r$r.log; exit 1; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(f'{sys.argv[2]:>14} r{sys.argv[3]} {sys.argv[4]:>9} envs  step {r[\"kernel_ms_mean\"]*1e3:7.2f} us  frac {r[\"frac\"]:.3f}')" \
        gpurun_out/abs/${tag}_${e}_r$r.log "$tag" "$r" "$e"
    done
  done
done
