set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== qnet tests" && { timeout -k 10 600 python -m pytest tests/test_gpu_qnet.py -x -q > gpurun_out/pytest_qnet.log 2>&1; rc=$?; tail -30 gpurun_out/pytest_qnet.log; [ $rc -eq 0 ]; } \
&& echo "== all gpu tests" && { timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ]; } \
&& echo "== bench" && timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log
