# r05f: config-5 self / other through the round-5 pass structure with all envs listed (allneed), and
# isolation variants: q1 inputs without the list read, q2 + compile-time view per chunk, q3 + scatter
# without the list read, q4 the round-4 Q-net waves with the round-5 env waves
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05f
mkdir -p $O
L="tools/variants/lib_r05base.so tools/variants/lib_allneed.so tools/variants/lib_q1.so tools/variants/lib_q2.so tools/variants/lib_q3.so tools/variants/lib_q4.so"
echo "== ab qnet" && timeout -k 10 600 python tools/ab_kernels.py --qnet $L > $O/ab_qnet.log 2>&1; rc=$?; tail -6 $O/ab_qnet.log; exit $rc
