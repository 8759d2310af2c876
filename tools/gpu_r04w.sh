# r04w: the policy kernels' statistics over many launches (new test) and a bench run after the
# bench.py formatting change.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04w
mkdir -p $O
echo "== pytest policy statistics" && timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_policy_statistics.py > $O/pytest_policy_stats.log 2>&1 && grep -E "policy statistics|passed|failed" $O/pytest_policy_stats.log \
&& echo "== bench k20" && timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20.log 2>&1 && tail -1 $O/bench_k20.log | cut -c1-150 \
&& echo "== all ok"
