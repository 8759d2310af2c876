# bench.py's rollout leg under different preambles (same box): kernel us per env-step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
run() { timeout -k 10 200 python bench.py --no-cpu-baseline --qnet-launches 0 --replay-stores 0 "$@" > gpurun_out/bcmp.log 2>&1 \
  && python -c "import json,sys; d=json.loads(open('gpurun_out/bcmp.log').read().strip().splitlines()[-1]); print(sys.argv[1:], 'rollout us/step %.2f' % (d['rollout']['kernel_ms_mean']*1e3/16), 'step us %.2f' % (d['roofline']['kernel_ms_mean']*1e3))" "$@"; }
run && run --no-events && run --steps 100 && run --rollout-launches 200 && run --steps 3000
