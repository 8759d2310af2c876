# r04z: which half of the env-wave change gains on config 5 -- the LDS action_dict table in the
# lockstep step (lib_qlds) or the by-value cold sincos (lib_sincos) -- against the product build and
# the two together (lib_envwave_nw); the rollout with the cold sincos change alone.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04z
mkdir -p $O
V="tools/variants/lib_rp_base.so tools/variants/lib_qlds.so tools/variants/lib_sincos.so tools/variants/lib_envwave_nw.so"
echo "== ab qnet" && MG_AB_FLAGS=1 timeout -k 10 500 python tools/ab_kernels.py $V --qnet --rounds 5 --warm 1200 > $O/ab_qnet.log 2>&1 && tail -4 $O/ab_qnet.log \
&& echo "== ab qnet rev" && MG_AB_FLAGS=1 timeout -k 10 500 python tools/ab_kernels.py tools/variants/lib_envwave_nw.so tools/variants/lib_sincos.so tools/variants/lib_qlds.so tools/variants/lib_rp_base.so --qnet --rounds 5 --warm 1200 > $O/ab_qnet_rev.log 2>&1 && tail -4 $O/ab_qnet_rev.log \
&& echo "== ab rollout" && MG_AB_FLAGS=1 timeout -k 10 400 python tools/ab_kernels.py tools/variants/lib_rp_base.so tools/variants/lib_sincos.so --rounds 8 --warm 1200 --rollouts 8 > $O/ab_rollout.log 2>&1 && tail -3 $O/ab_rollout.log | head -2 \
&& echo "== all ok"
