set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== qnet+replay tests" && { timeout -k 10 400 python -u -m pytest tests/test_gpu_qnet.py tests/test_gpu_replay.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_qnet.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_qnet.log; [ $rc -eq 0 ]; } \
&& echo "== ab qnet" && timeout -k 10 300 python tools/ab_kernels.py merging-gym_amd/variants/lib_*.so --qnet --rounds 5 --warm 1200 > gpurun_out/ab_qnet.log 2>&1; tail -5 gpurun_out/ab_qnet.log
