# Q-net forward check: the Q-net / h-DQN / packing GPU tests, then the default bench (its Q-net and
# h-DQN legs). Every GPU step has its own time limit; the chain stops at the first failure.
# Usage: TAG=r03ac bash tools/gpu_r03q.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r03q}
O=gpurun_out/$TAG
mkdir -p $O
echo "== pytest qnet" && { timeout -k 10 600 python -u -m pytest tests/test_gpu_qnet_fragments.py tests/test_gpu_qnet.py tests/test_gpu_hdqn.py tests/test_gpu_hdqn_reset.py -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_qnet.log 2>&1; rc=$?; tail -3 $O/pytest_qnet.log; [ $rc -eq 0 ]; } \
&& echo "== ab qnet" && timeout -k 10 300 python tools/ab_kernels.py tools/variants/lib_*.so --qnet --rounds 5 --warm 1200 > $O/ab_qnet.log 2>&1 && tail -4 $O/ab_qnet.log \
&& echo "== ab hdqn" && timeout -k 10 400 python tools/ab_hdqn.py tools/variants/lib_*.so > $O/ab_hdqn.log 2>&1 && tail -3 $O/ab_hdqn.log \
&& echo "== bench default" && timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_default.log 2>&1 && tail -1 $O/bench_default.log | cut -c1-300 \
&& echo "== all ok"
