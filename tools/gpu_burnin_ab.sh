# Does the burn-in's kernel (fused rollouts vs one-step launches; the env state at the window is
# the same either way: Philox actions keyed by env and step) change the step kernel's timed
# window? Step leg only, K=300 and the driver's K=20, interleaved over ROUNDS rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/burnin
mkdir -p $O
COMMON="--no-cpu-baseline --qnet-launches 0 --replay-stores 0 --rollout-steps 0 --size2-envs 0"
for r in $(seq 1 ${ROUNDS:-3}); do
  for mode in rollout steps; do
    if [ $mode = rollout ]; then B="--burn-in 1024 --burn-in-launches 48"; else B="--burn-in 0 --burn-in-launches 1072"; fi  # the shipped default since this A/B
    for K in 300 20; do
      W=10; [ $K = 20 ] && W=5
      timeout -k 10 180 python bench.py --steps $K --warmup $W $B $COMMON > $O/${mode}_k${K}_r$r.log 2>&1 || { echo "$mode $K failed"; tail -3 $O/${mode}_k${K}_r$r.log; exit 1; }
      python - $mode $K $r $O/${mode}_k${K}_r$r.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[4]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[1]:>8} K={sys.argv[2]:>3} r{sys.argv[3]}  value {d['value']:.4e}  kernel {r['kernel_ms_mean']*1e3:6.2f} us  "
      f"ms/step {d['ms_per_step']*1e3:6.2f} us  episodes {d['episodes'].get('completed')}")
PY
    done
  done
done
