# r05g: h-DQN and config-5 (opponent modes 2 / 3) kernels with compacted forwards on compile-time
# column counts (qnet_mlp_nc): the policy GPU tests, then in-process A/Bs against the round-4 library
# (tools/variants/lib_r05base.so, built from HEAD)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05g
mkdir -p $O
echo "== ab hdqn" && timeout -k 10 400 python tools/ab_hdqn.py tools/variants/lib_r05base.so merging-gym_amd/merging_gym/libmerging_hip.so --rounds 3 > $O/ab_hdqn.log 2>&1; rc=$?; tail -2 $O/ab_hdqn.log; [ $rc -eq 0 ] || exit $rc
echo "== ab qnet" && timeout -k 10 400 python tools/ab_kernels.py --qnet tools/variants/lib_r05base.so merging-gym_amd/merging_gym/libmerging_hip.so > $O/ab_qnet.log 2>&1; rc=$?; tail -2 $O/ab_qnet.log; [ $rc -eq 0 ] || exit $rc
echo "== pytest policy" && timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_hdqn.py tests/test_gpu_hdqn_reset.py tests/test_gpu_qnet.py tests/test_gpu_policy_statistics.py > $O/pytest_policy.log 2>&1; rc=$?; tail -3 $O/pytest_policy.log; exit $rc
