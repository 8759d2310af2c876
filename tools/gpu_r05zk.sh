# r05zk: run-to-run determinism of the config-5 and h-DQN kernels (tests/test_gpu_determinism.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05zk
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_determinism.py > $O/pytest.log 2>&1; rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest.log | tail -8; exit $rc
