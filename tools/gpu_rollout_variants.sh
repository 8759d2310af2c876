# bench.py's rollout leg (T = 16, 10 + 200 launches) and config-5 Q-net leg for each variant library, interleaved,
# after the GPU test suite on the in-tree build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
echo "== pytest gpu" && { timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ]; } || exit 1
V=merging-gym_amd/variants
for rep in 1 2 3; do for lib in $V/lib_*.so; do
  MERGING_HIP_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 200 --no-cpu-baseline --replay-stores 0 > gpurun_out/brv.log 2>&1 || { tail -5 gpurun_out/brv.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/brv.log').read().strip().splitlines()[-1]); r=d['rollout']; q=d['qnet_policy']; print(sys.argv[1], 'rollout %.4e' % r['value'], 'kernel us/step %.3f' % (r['kernel_ms_mean']*1e3/16), 'qnet ego %.4e self %.4e' % (q[0]['value'], q[1]['value']), 'step %.2f us' % (d['roofline']['kernel_ms_mean']*1e3))" $(basename $lib)
done; done
