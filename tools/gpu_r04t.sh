# r04t: h-DQN with the opponent's nets in the env waves as two 32-env half forwards
# (qnet_mlp_half; lib_half_mem = the working tree, env state in memory between steps; lib_half_reg
# the env state in registers): parity on the working tree, then the A/B against the committed build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04t
mkdir -p $O
echo "== pytest hdqn" && timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_hdqn.py tests/test_gpu_hdqn_reset.py > $O/pytest_hdqn.log 2>&1 && tail -2 $O/pytest_hdqn.log \
&& echo "== ab hdqn" && timeout -k 10 400 python tools/ab_hdqn.py tools/variants/lib_rp_base.so tools/variants/lib_half_mem.so tools/variants/lib_half_reg.so > $O/ab_hdqn.log 2>&1 && tail -4 $O/ab_hdqn.log \
&& echo "== all ok"
