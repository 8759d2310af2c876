# A/B of the variant libraries in tools/variants: h-DQN legs (tools/ab_hdqn.py) and config-5 legs
# (tools/ab_kernels.py --qnet). Usage: TAG=r03ah bash tools/gpu_r03ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r03ab}
O=gpurun_out/$TAG
mkdir -p $O
echo "== ab hdqn" && timeout -k 10 400 python tools/ab_hdqn.py tools/variants/lib_*.so > $O/ab_hdqn.log 2>&1 && tail -4 $O/ab_hdqn.log \
&& echo "== ab qnet" && timeout -k 10 300 python tools/ab_kernels.py tools/variants/lib_*.so --qnet --rounds 8 --warm 1200 > $O/ab_qnet.log 2>&1 && tail -4 $O/ab_qnet.log \
&& echo "== all ok"
