# r04y: the replay store with every load landed before the first row store (no store drain between
# steps; lib_rp_land2 = the working tree, rp_land4: 4 steps per write block) against the product
# build: parity, then the A/B in both orders.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04y
mkdir -p $O
echo "== pytest replay" && timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_replay.py > $O/pytest_replay.log 2>&1 && tail -2 $O/pytest_replay.log \
&& echo "== ab replay" && timeout -k 10 300 python tools/ab_kernels.py tools/variants/lib_rp_base.so tools/variants/lib_rp_land2.so tools/variants/lib_rp_land4.so --replay --rounds 8 > $O/ab_replay.log 2>&1 && tail -3 $O/ab_replay.log \
&& echo "== ab replay rev" && timeout -k 10 300 python tools/ab_kernels.py tools/variants/lib_rp_land4.so tools/variants/lib_rp_land2.so tools/variants/lib_rp_base.so --replay --rounds 8 > $O/ab_replay_rev.log 2>&1 && tail -3 $O/ab_replay_rev.log \
&& echo "== ab rollout (no vector loads in the step loop)" && MG_AB_FLAGS=1 timeout -k 10 400 python tools/ab_kernels.py tools/variants/lib_rp_base.so tools/variants/lib_roll_nw.so --rounds 8 --warm 1200 --rollouts 8 > $O/ab_rollout.log 2>&1 && tail -3 $O/ab_rollout.log | head -2 \
&& echo "== ab rollout rev" && MG_AB_FLAGS=1 timeout -k 10 400 python tools/ab_kernels.py tools/variants/lib_roll_nw.so tools/variants/lib_rp_base.so --rounds 8 --warm 1200 --rollouts 8 > $O/ab_rollout_rev.log 2>&1 && tail -3 $O/ab_rollout_rev.log | head -2 \
&& echo "== ab qnet (env waves without vector loads)" && MG_AB_FLAGS=1 timeout -k 10 400 python tools/ab_kernels.py tools/variants/lib_rp_base.so tools/variants/lib_envwave_nw.so --qnet --rounds 5 --warm 1200 > $O/ab_qnet.log 2>&1 && tail -2 $O/ab_qnet.log \
&& echo "== ab hdqn" && timeout -k 10 400 python tools/ab_hdqn.py tools/variants/lib_rp_base.so tools/variants/lib_envwave_nw.so > $O/ab_hdqn.log 2>&1 && tail -2 $O/ab_hdqn.log \
&& echo "== all ok"
