# In-process A/B of tools/variants/lib_*.so: step + rollout (interleaved record), config-5 Q-net, h-DQN.
# Usage: TAG=r04x LIBS="tools/variants/lib_a.so tools/variants/lib_b.so" bash tools/gpu_r04ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r04ab}
O=gpurun_out/$TAG
mkdir -p $O
LIBS=${LIBS:-tools/variants/lib_*.so}
echo "== ab step/rollout" && MG_AB_FLAGS=1 timeout -k 10 300 python tools/ab_kernels.py $LIBS --rounds 6 --warm 1200 > $O/ab_rollout.log 2>&1 && tail -4 $O/ab_rollout.log \
&& echo "== ab qnet" && timeout -k 10 300 python tools/ab_kernels.py $LIBS --qnet --rounds 5 --warm 1200 > $O/ab_qnet.log 2>&1 && tail -8 $O/ab_qnet.log \
&& echo "== ab hdqn" && timeout -k 10 400 python tools/ab_hdqn.py $LIBS --rounds 4 > $O/ab_hdqn.log 2>&1 && tail -8 $O/ab_hdqn.log \
&& echo "== ab ok"
