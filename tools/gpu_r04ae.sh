#!/bin/bash
# r04ae: h-DQN goal outputs (goal, goal_op, next_goal, reward) and q_eval atomics moved from the
# Q-net waves to the env waves: parity (h-DQN + statistics GPU tests), then the A/B against the
# previous product (lib_sc.so) in both orders.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ae
mkdir -p $O
echo "== hdqn tests" && timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_hdqn.py tests/test_gpu_hdqn_reset.py tests/test_gpu_policy_statistics.py tests/test_gpu_replay.py > $O/pytest_hdqn.log 2>&1 && tail -2 $O/pytest_hdqn.log \
&& echo "== ab hdqn" && timeout -k 10 400 python tools/ab_hdqn.py tools/variants/lib_sc.so tools/variants/lib_hgoals.so --rounds 6 > $O/ab_hdqn.log 2>&1 && tail -4 $O/ab_hdqn.log \
&& echo "== ab hdqn rev" && timeout -k 10 400 python tools/ab_hdqn.py tools/variants/lib_hgoals.so tools/variants/lib_sc.so --rounds 6 > $O/ab_hdqn_rev.log 2>&1 && tail -4 $O/ab_hdqn_rev.log \
&& echo "== all ok"
