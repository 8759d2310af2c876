# r05za: config-5 rollout test with every env's clock three steps short of the timeout (sync cases)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05za
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_qnet.py -k "policy_and_transitions" > $O/pytest.log 2>&1; rc=$?; grep -E "PASSED|FAILED|ERROR|near-tie|q_eval" $O/pytest.log | tail -20; exit $rc
