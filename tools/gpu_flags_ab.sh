# bench.py step leg with the interleaved step record (MG_STEP_FLAGS=1, default) vs four byte
# arrays (MG_STEP_FLAGS=0), interleaved runs on one box, after the GPU test suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
echo "== pytest gpu" && { timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ]; } || exit 1
for e in 1048576 4194304; do for rep in 1 2 3; do for fl in 0 1; do
  MG_STEP_FLAGS=$fl timeout -k 10 200 python bench.py --envs $e --steps 1000 --warmup 1000 --no-cpu-baseline --rollout-steps 0 --qnet-launches 0 --replay-stores 0 > gpurun_out/fa.log 2>&1 || { tail -5 gpurun_out/fa.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/fa.log').read().strip().splitlines()[-1]); r=d['roofline']; print('envs', sys.argv[1], 'flags', sys.argv[2], '%.4e' % d['value'], 'kernel %.2f us' % (r['kernel_ms_mean']*1e3), 'dispatch %.2f us' % (r['kernel_ms_dispatch_sample']*1e3), 'frac %.3f' % r['frac'])" $e $fl
done; done; done
