# GPU tests, then the rollout with separate byte arrays vs the interleaved flags buffer (same library).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
V=merging-gym_amd/variants
echo "== pytest gpu" && { timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ]; } \
&& for f in 0 1 0 1; do MG_AB_FLAGS=$f timeout -k 10 200 python tools/ab_kernels.py $V/lib_new.so --rounds 4 --warm 1000 2>&1 | grep "lib_" | sed "s/^/flags=$f /" | cut -c1-200 || exit 1; done \
&& for f in 0 1; do MG_AB_FLAGS=$f timeout -k 10 200 python tools/ab_kernels.py $V/lib_new.so --qnet --rounds 3 --warm 1200 2>&1 | grep "lib_" | sed "s/^/flags=$f /" || exit 1; done
