# r05zm: config-5 actions outside action_dict with the other-net opponent (net-split kernel)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05zm
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_qnet.py -k invalid_greedy > $O/pytest.log 2>&1; rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest.log | tail -5; exit $rc
