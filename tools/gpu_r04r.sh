# r04r: the random rollout's counts added with no-return atomics at the launch end (lib_cnt_atomic)
# against the product build; in-process A/B in both orders.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04r
mkdir -p $O
echo "== ab rollout" && MG_AB_FLAGS=1 timeout -k 10 400 python tools/ab_kernels.py tools/variants/lib_rp_base.so tools/variants/lib_cnt_atomic.so --rounds 10 --warm 1200 --rollouts 8 > $O/ab_rollout.log 2>&1 && tail -3 $O/ab_rollout.log | head -2 \
&& echo "== ab rollout rev" && MG_AB_FLAGS=1 timeout -k 10 400 python tools/ab_kernels.py tools/variants/lib_cnt_atomic.so tools/variants/lib_rp_base.so --rounds 10 --warm 1200 --rollouts 8 > $O/ab_rollout_rev.log 2>&1 && tail -3 $O/ab_rollout_rev.log | head -2 \
&& echo "== all ok"
