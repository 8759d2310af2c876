# One build variant on the GPU: the step / rollout / Q-net parity tests against it, then the
# bench legs A/B against the shipped library. Usage: ROUNDS=2 bash tools/gpu_variant_check.sh tools/variants/lib_x.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/variant
mkdir -p $O
LIB=$1
echo "== parity ($LIB)" && { MERGING_HIP_LIB=$PWD/$LIB timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_dropin.py tests/test_gpu_qnet.py tests/test_gpu_hdqn.py} -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ]; } \
&& echo "== A/B" && ROUNDS=${ROUNDS:-2} bash tools/gpu_ab_legs.sh "$LIB" 2>&1 | tee $O/ab.txt \
&& echo "== all ok"
