# r04q: the random rollout with its statistics read lazily (lib_lazy = the working tree) against the
# product build: parity (rollout = step sequence, records) and the in-process A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04q
mkdir -p $O
echo "== pytest" && timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_episode_stats.py tests/test_gpu_distributed.py tests/test_gpu_replay.py > $O/pytest.log 2>&1 && tail -2 $O/pytest.log \
&& echo "== ab rollout" && MG_AB_FLAGS=1 timeout -k 10 400 python tools/ab_kernels.py tools/variants/lib_rp_base.so tools/variants/lib_lazy.so --rounds 10 --warm 1200 --rollouts 8 > $O/ab_rollout.log 2>&1 && tail -3 $O/ab_rollout.log | head -2 \
&& echo "== ab rollout rev" && MG_AB_FLAGS=1 timeout -k 10 400 python tools/ab_kernels.py tools/variants/lib_lazy.so tools/variants/lib_rp_base.so --rounds 10 --warm 1200 --rollouts 8 > $O/ab_rollout_rev.log 2>&1 && tail -3 $O/ab_rollout_rev.log | head -2 \
&& echo "== all ok"
