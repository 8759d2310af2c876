# Layer-2 tail on 4x4x4 MFMAs (MG_QNET_TAIL4): operand-layout probe, MFMA issue rates, the
# Q-net / h-DQN GPU parity tests against the tail build, then the config-5 / h-DQN A/B against
# the shipped library. Every GPU step has its own time limit; the chain stops at the first failure.
# Usage (on the GPU box): bash tools/gpu_tail4.sh tools/variants/lib_tail4.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/tail4
mkdir -p $O
LIB=$1
echo "== layout" && timeout -k 10 60 ./tools/micro/mfma4_layout | tee $O/layout.txt \
&& echo "== mfma rate" && timeout -k 10 60 ./tools/micro/mfma_rate | tee $O/mfma_rate.txt \
&& echo "== parity (tail build)" && { MERGING_HIP_LIB=$PWD/$LIB timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_qnet.py tests/test_gpu_hdqn.py} -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ]; } \
&& echo "== A/B" && ROUNDS=${ROUNDS:-2} bash tools/gpu_qnet_ab.sh "$LIB" 2>&1 | tee $O/ab.txt \
&& echo "== all ok"
