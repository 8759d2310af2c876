# Headline step leg at several batch sizes (one bench line each): where the GPU saturates.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
: > gpurun_out/size_sweep.jsonl
for e in 65536 262144 1048576 4194304 8388608 16777216; do
  timeout -k 10 200 python bench.py --envs $e --steps 300 --no-cpu-baseline --rollout-steps 0 --qnet-launches 0 --replay-stores 0 > gpurun_out/bs.log 2>&1 || { tail -5 gpurun_out/bs.log; exit 1; }
  tail -1 gpurun_out/bs.log >> gpurun_out/size_sweep.jsonl
  python -c "import json; d=json.loads(open('gpurun_out/bs.log').read().strip().splitlines()[-1]); r=d['roofline']; print(d['config']['envs_per_gpu'], '%.3e' % d['value'], 'kernel %.2f us' % (r['kernel_ms_mean']*1e3), 'dispatch %.2f us' % (r['kernel_ms_dispatch_sample']*1e3), 'frac %.3f' % r['frac'])"
done
