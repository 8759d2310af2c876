# r05zo: closing A/B of the round-4 library (rebuilt from its source) against the final round-5
# library, config 5 and h-DQN, more rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05zo
mkdir -p $O
echo "== ab qnet" && timeout -k 10 600 python tools/ab_kernels.py --qnet tools/variants/lib_r04.so merging-gym_amd/merging_gym/libmerging_hip.so --rounds 12 > $O/ab_qnet.log 2>&1 && tail -2 $O/ab_qnet.log \
&& echo "== ab hdqn" && timeout -k 10 600 python tools/ab_hdqn.py tools/variants/lib_r04.so merging-gym_amd/merging_gym/libmerging_hip.so --rounds 6 > $O/ab_hdqn.log 2>&1 && tail -2 $O/ab_hdqn.log
