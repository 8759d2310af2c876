# r05x: h-DQN lower passes compacted (48 items on the Q-net waves, the rest on the env waves): GPU tests, A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05x
mkdir -p $O
echo "== pytest hdqn" && timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hdqn.py tests/test_gpu_episode_stats.py > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
echo "== ab hdqn" && timeout -k 10 600 python tools/ab_hdqn.py tools/variants/lib_r05base.so tools/variants/lib_r05c.so merging-gym_amd/merging_gym/libmerging_hip.so tools/variants/lib_hd_low3.so --rounds 4 > $O/ab_hdqn.log 2>&1; rc=$?; tail -4 $O/ab_hdqn.log; exit $rc
