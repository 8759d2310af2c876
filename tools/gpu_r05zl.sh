# r05zl: checkpoint / resume GPU tests after load_state_dict restores absent h-DQN state as none
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05zl
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_hdqn.py tests/test_gpu_hdqn_reset.py tests/test_gpu_determinism.py > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; exit $rc
