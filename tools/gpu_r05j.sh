# r05j: fragment ring deepened for narrow forwards (qnet_mlp_nc): A/B against the round-4 library
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05j
mkdir -p $O
echo "== ab hdqn" && timeout -k 10 400 python tools/ab_hdqn.py tools/variants/lib_r05base.so merging-gym_amd/merging_gym/libmerging_hip.so --rounds 3 > $O/ab_hdqn.log 2>&1; rc=$?; tail -2 $O/ab_hdqn.log; [ $rc -eq 0 ] || exit $rc
echo "== ab qnet" && timeout -k 10 400 python tools/ab_kernels.py --qnet tools/variants/lib_r05base.so merging-gym_amd/merging_gym/libmerging_hip.so > $O/ab_qnet.log 2>&1; rc=$?; tail -2 $O/ab_qnet.log; exit $rc
