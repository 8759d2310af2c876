# h-DQN / config-5 legs of bench.py for the shipped library and each variant given, interleaved
# over ROUNDS rounds on one box. Usage: ROUNDS=2 bash tools/gpu_ab_hdqn.sh tools/variants/lib_x.so ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abh
ROUNDS=${ROUNDS:-2}
for r in $(seq 1 "$ROUNDS"); do
  for lib in default "$@"; do
    tag=$(basename "$lib" .so)
    if [ "$lib" = default ]; then unset MERGING_HIP_LIB; else export MERGING_HIP_LIB=$PWD/$lib; fi
    timeout -k 10 240 python bench.py --steps 100 --warmup 10 --burn-in 320 --rollout-launches 50 \
      --replay-stores 0 --size2-envs 0 --no-cpu-baseline > gpurun_out/abh/${tag}_r$r.log 2>&1 || { echo "$tag failed"; tail -3 gpurun_out/abh/${tag}_r$r.log; exit 1; }
    python - "$tag" "$r" gpurun_out/abh/${tag}_r$r.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
q, h = d["qnet_policy"], d["hdqn_policy"]
print(f"{sys.argv[1]:>16} r{sys.argv[2]}  qnet ego {q[0]['kernel_ms_mean']:.3f} self {q[1]['kernel_ms_mean']:.3f} "
      f"other {q[2]['kernel_ms_mean']:.3f} ms  hdqn {h['kernel_ms_mean']:.3f} self {h['selfplay']['kernel_ms_mean']:.3f} "
      f"other {h['other_checkpoint']['kernel_ms_mean']:.3f} ms per 16-step launch")
PY
  done
done
