# r05o: config-5 role ablation (noq: the Q-net waves skip their forwards; noenv: the env waves skip
# their steps) beside the round-4 and round-5 libraries; the chunked long-rollout test
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05o
mkdir -p $O
echo "== pytest chunked rollout" && timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k chunked > $O/pytest_chunk.log 2>&1; rc=$?; tail -2 $O/pytest_chunk.log; [ $rc -eq 0 ] || exit $rc
echo "== ab qnet roles" && timeout -k 10 500 python tools/ab_kernels.py --qnet tools/variants/lib_r05base.so merging-gym_amd/merging_gym/libmerging_hip.so tools/variants/lib_noq.so tools/variants/lib_noenv.so > $O/ab_roles.log 2>&1; rc=$?; tail -4 $O/ab_roles.log; exit $rc
