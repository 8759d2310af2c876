# Leg warm-up A/B: bench.py --leg-warmup 10 (shipped) vs 60 for the rollout, Q-net and h-DQN legs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/legwarm
for r in 1 2; do for lw in 10 60; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 --leg-warmup $lw --replay-stores 0 --size2-envs 0 --no-cpu-baseline > gpurun_out/legwarm/lw${lw}_r$r.log 2>&1 || exit 1
  python - $lw $r gpurun_out/legwarm/lw${lw}_r$r.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1]); q = d["qnet_policy"]; h = d["hdqn_policy"]
print(f"leg-warmup {sys.argv[1]:>3} r{sys.argv[2]}  rollout {d['rollout']['kernel_ms_mean']*1e3/16:6.2f}  qnet {q[0]['kernel_ms_mean']*1e3/16:6.2f} {q[1]['kernel_ms_mean']*1e3/16:6.2f} {q[2]['kernel_ms_mean']*1e3/16:6.2f}  hdqn {h['kernel_ms_mean']*1e3/16:6.2f} us/step")
PY
done; done
