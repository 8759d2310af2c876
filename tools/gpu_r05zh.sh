# r05zh: h-DQN Q-net waves lower passes listed by the env waves, 48 per Q-net wave, the rest on env waves 0 and 1: GPU tests, A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05zh
mkdir -p $O
echo "== pytest hdqn" && timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hdqn.py tests/test_gpu_episode_stats.py tests/test_gpu_policy_statistics.py > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
echo "== ab hdqn" && timeout -k 10 600 python tools/ab_hdqn.py tools/variants/lib_r05base.so tools/variants/lib_r05e.so merging-gym_amd/merging_gym/libmerging_hip.so --rounds 5 > $O/ab_hdqn.log 2>&1; rc=$?; tail -3 $O/ab_hdqn.log; exit $rc
