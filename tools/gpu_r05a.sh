# r05a: the h-DQN kernel with compacted forwards (greedy branches only): its GPU tests, then an
# in-process A/B against the round-4 library (tools/variants/lib_r05base.so, built from HEAD)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05a
mkdir -p $O
echo "== pytest hdqn" && timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_hdqn.py tests/test_gpu_hdqn_reset.py > $O/pytest_hdqn.log 2>&1; rc=$?; tail -3 $O/pytest_hdqn.log; [ $rc -eq 0 ] || exit $rc
echo "== ab" && timeout -k 10 400 python tools/ab_hdqn.py tools/variants/lib_r05base.so merging-gym_amd/merging_gym/libmerging_hip.so --rounds 3 > $O/ab.log 2>&1; rc=$?; cat $O/ab.log | tail -5; exit $rc
