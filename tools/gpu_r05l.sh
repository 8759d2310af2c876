# r05l: config-5 self-play with staged fragments and merged lists: A/B + config-5 GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05l
mkdir -p $O
echo "== ab qnet" && timeout -k 10 400 python tools/ab_kernels.py --qnet tools/variants/lib_r05base.so merging-gym_amd/merging_gym/libmerging_hip.so --rounds 7 > $O/ab_qnet.log 2>&1; rc=$?; tail -2 $O/ab_qnet.log; [ $rc -eq 0 ] || exit $rc
echo "== pytest qnet" && timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_qnet.py tests/test_gpu_policy_statistics.py > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; exit $rc
