# Step / rollout / config-5 legs of bench.py for the shipped library and each variant given,
# interleaved over ROUNDS rounds (same box). Usage: ROUNDS=2 bash tools/gpu_ab_legs.sh tools/variants/lib_x.so ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abl
ROUNDS=${ROUNDS:-2}
for r in $(seq 1 "$ROUNDS"); do
  for lib in default "$@"; do
    tag=$(basename "$lib" .so)
    if [ "$lib" = default ]; then unset MERGING_HIP_LIB; else export MERGING_HIP_LIB=$PWD/$lib; fi
    timeout -k 10 240 python bench.py --steps 300 --warmup 10 --burn-in 320 --rollout-launches 100 \
      --replay-stores 0 --size2-envs 0 --no-cpu-baseline > gpurun_out/abl/${tag}_r$r.log 2>&1 || { echo "$tag failed"; tail -3 gpurun_out/abl/${tag}_r$r.log; exit 1; }
    python - "$tag" "$r" gpurun_out/abl/${tag}_r$r.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
q = d["qnet_policy"]
print(f"{sys.argv[1]:>16} r{sys.argv[2]}  step {d['roofline']['kernel_ms_mean']*1e3:6.2f} us  rollout "
      f"{d['rollout']['kernel_ms_mean']*1e3/16:6.2f} us/step ({d['rollout']['value']:.3e})  qnet ego {q[0]['kernel_ms_mean']*1e3/16:6.2f} "
      f"self {q[1]['kernel_ms_mean']*1e3/16:6.2f}  hdqn {d['hdqn_policy']['kernel_ms_mean']*1e3/16:6.2f} us/step")
PY
  done
done
