# Driver-style short windows (K = 20, W = 5) with and without hipDeviceScheduleSpin, 3 rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/win
for r in 1 2 3; do
  for spin in 1 0; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --sync-spin $spin --no-cpu-baseline --size2-envs 0 \
      --rollout-steps 0 > gpurun_out/win/k20_spin${spin}_r$r.log 2>&1 || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], round(d['ms_per_step']*1e3,2), round(r['kernel_ms_mean']*1e3,2), round(r['wall_over_kernel'],4), round(r['host_enqueue_ms_per_launch']*1e3,2), r['host_sync'])" gpurun_out/win/k20_spin${spin}_r$r.log "spin=$spin r$r"
  done
done
