# bench.py step leg with the staggered arena (default) vs separate allocations, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
echo "== pytest gpu" && { timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ]; } || exit 1
for e in 1048576 8388608; do for rep in 1 2 3; do for st in -1 4160; do
  MG_ARENA_STAGGER=$st timeout -k 10 200 python bench.py --envs $e --steps 400 --no-cpu-baseline --rollout-steps 0 --qnet-launches 0 --replay-stores 0 > gpurun_out/ba.log 2>&1 || { tail -5 gpurun_out/ba.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/ba.log').read().strip().splitlines()[-1]); print('envs', sys.argv[1], 'stagger', sys.argv[2], '%.4e' % d['value'], 'kernel %.2f us' % (d['roofline']['kernel_ms_mean']*1e3), 'frac %.3f' % d['roofline']['frac'])" $e $st
done; done; done
