# r05zj: config-5 L0 / uniform-opponent kernel with both tiles' inputs read at the phase start: GPU tests, A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05zj
mkdir -p $O
echo "== pytest qnet" && timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_qnet.py tests/test_gpu_policy_statistics.py > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
echo "== ab qnet" && timeout -k 10 600 python tools/ab_kernels.py --qnet tools/variants/lib_r05base.so tools/variants/lib_r05f.so merging-gym_amd/merging_gym/libmerging_hip.so --rounds 8 > $O/ab_qnet.log 2>&1; rc=$?; tail -3 $O/ab_qnet.log; exit $rc
