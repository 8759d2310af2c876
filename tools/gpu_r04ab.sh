# r04ab: the rollout with the by-value cold sincos (lib_sc = the working tree) against the build
# before it, longer, both orders.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04ab
mkdir -p $O
echo "== ab rollout" && MG_AB_FLAGS=1 timeout -k 10 500 python tools/ab_kernels.py tools/variants/lib_rp_base.so tools/variants/lib_sc.so tools/variants/lib_sc_split.so --rounds 12 --warm 1200 --rollouts 8 > $O/ab_rollout.log 2>&1 && tail -4 $O/ab_rollout.log | head -3 \
&& echo "== ab rollout rev" && MG_AB_FLAGS=1 timeout -k 10 500 python tools/ab_kernels.py tools/variants/lib_sc_split.so tools/variants/lib_sc.so tools/variants/lib_rp_base.so --rounds 12 --warm 1200 --rollouts 8 > $O/ab_rollout_rev.log 2>&1 && tail -4 $O/ab_rollout_rev.log | head -3 \
&& echo "== ab qnet" && MG_AB_FLAGS=1 timeout -k 10 400 python tools/ab_kernels.py tools/variants/lib_rp_base.so tools/variants/lib_sc.so tools/variants/lib_sc_split.so --qnet --rounds 4 --warm 1200 > $O/ab_qnet.log 2>&1 && tail -3 $O/ab_qnet.log \
&& echo "== all ok"
