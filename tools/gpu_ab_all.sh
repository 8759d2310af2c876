# GPU tests with the in-tree library, then A/B of the variant libraries (step, rollout, Q-net).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
V=merging-gym_amd/variants
echo "== pytest gpu" && { timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ]; } \
&& echo "== ab step/rollout" && timeout -k 10 300 python tools/ab_kernels.py $V/lib_*.so --rounds 8 --warm 1000 > gpurun_out/ab1.log 2>&1 && grep -v amdgpu.ids gpurun_out/ab1.log | grep -v '^{' | cut -c1-230 \
&& echo "== ab qnet" && timeout -k 10 300 python tools/ab_kernels.py $V/lib_*.so --qnet --rounds 5 --warm 1200 > gpurun_out/ab_qnet.log 2>&1; grep -v amdgpu.ids gpurun_out/ab_qnet.log
