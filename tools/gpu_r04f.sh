# r04f: rollout twin (with the two-envs-per-lane pattern), default and driver-style bench with the
# staggered burn-in (no 2^22 rehearsal window), rocprofv3 stats of the default bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04f
mkdir -p $O
echo "== rollout twin" && timeout -k 10 120 ./tools/micro/rollout_twin > $O/rollout_twin.txt && cat $O/rollout_twin.txt \
&& echo "== bench default" && timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 && tail -1 $O/bench_default.log | cut -c1-200 \
&& echo "== bench driver-style" && timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20.log 2>&1 && tail -1 $O/bench_k20.log | cut -c1-200 \
&& echo "== rocprof stats" && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o r04f -- python bench.py --no-cpu-baseline > $O/prof.log 2>&1 \
&& echo "== all ok"
