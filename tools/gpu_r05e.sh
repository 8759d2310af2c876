# r05e: A/B of round-4 library / allneed / envold (allneed with the env waves drawing at step time,
# no draws one phase ahead and no may-finish predicate)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05e
mkdir -p $O
L="tools/variants/lib_r05base.so tools/variants/lib_allneed.so tools/variants/lib_envold.so"
echo "== ab hdqn" && timeout -k 10 500 python tools/ab_hdqn.py $L --rounds 2 > $O/ab_hdqn.log 2>&1; rc=$?; tail -3 $O/ab_hdqn.log; [ $rc -eq 0 ] || exit $rc
echo "== ab qnet" && timeout -k 10 500 python tools/ab_kernels.py --qnet $L > $O/ab_qnet.log 2>&1; rc=$?; tail -3 $O/ab_qnet.log; exit $rc
