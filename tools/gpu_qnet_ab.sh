# Config-5 A/B: bench.py's Q-net legs (ego / self-play, 10 untimed + 40 timed launches) for the
# shipped library and each tools/variants/lib_*.so given, interleaved over ROUNDS rounds.
# Usage (on the GPU box): ROUNDS=2 bash tools/gpu_qnet_ab.sh tools/variants/lib_a.so ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/qab
ROUNDS=${ROUNDS:-2}
for r in $(seq 1 "$ROUNDS"); do
  for lib in default "$@"; do
    tag=$(basename "$lib" .so)
    if [ "$lib" = default ]; then unset MERGING_HIP_LIB; else export MERGING_HIP_LIB=$PWD/$lib; fi
    timeout -k 10 240 python bench.py --steps 50 --warmup 5 --burn-in 320 --rollout-launches 40 \
      --replay-stores 0 --size2-envs 0 --no-cpu-baseline > gpurun_out/qab/${tag}_r$r.log 2>&1 || { echo "$tag failed"; exit 1; }
    python - "$tag" "$r" gpurun_out/qab/${tag}_r$r.log <<'EOF'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
q = d["qnet_policy"]
print(f"{sys.argv[1]:>14} r{sys.argv[2]}  step {d['roofline']['kernel_ms_mean']*1e3:6.2f} us  rollout "
      f"{d['rollout']['kernel_ms_mean']*1e3/16:6.2f} us/step  qnet ego {q[0]['kernel_ms_mean']*1e3/16:6.2f} "
      f"self {q[1]['kernel_ms_mean']*1e3/16:6.2f} us/step  frac {q[0]['frac_useful']:.3f} / {q[1]['frac_useful']:.3f}"
      + (f"  other-net {q[2]['kernel_ms_mean']*1e3/16:6.2f}" if len(q) > 2 else "")
      + (f"  hdqn {d['hdqn_policy']['kernel_ms_mean']*1e3/16:6.2f} self {d['hdqn_policy']['selfplay']['kernel_ms_mean']*1e3/16:6.2f}"
         if "hdqn_policy" in d else ""))
EOF
  done
done
