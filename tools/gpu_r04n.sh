# r04n: h-DQN with the opponent's nets in the env waves (lib_oppenv = the working tree) against the
# committed build: parity (the h-DQN GPU tests) first, then the in-process A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04n
mkdir -p $O
echo "== pytest hdqn" && timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_hdqn.py > $O/pytest_hdqn.log 2>&1 && tail -2 $O/pytest_hdqn.log \
&& echo "== ab hdqn" && timeout -k 10 400 python tools/ab_hdqn.py tools/variants/lib_nowait3.so tools/variants/lib_oppenv.so > $O/ab_hdqn.log 2>&1 && tail -3 $O/ab_hdqn.log \
&& echo "== all ok"
