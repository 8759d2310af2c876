# The headline bench line (step leg only) for each variant library, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
V=merging-gym_amd/variants
for rep in 1 2 3; do for lib in $V/lib_*.so; do
  MERGING_HIP_LIB=$PWD/$lib timeout -k 10 120 python bench.py --no-cpu-baseline --qnet-launches 0 --replay-stores 0 --rollout-steps 0 > gpurun_out/bv.log 2>&1 || { tail -5 gpurun_out/bv.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bv.log').read().strip().splitlines()[-1]); print(sys.argv[1], '%.4e' % d['value'], 'kernel %.2f us' % (d['roofline']['kernel_ms_mean']*1e3), 'wall %.2f us' % (d['ms_per_step']*1e3))" $(basename $lib)
done; done
