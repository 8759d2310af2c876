# r05c: where the compacted forwards lose time. A/B (one process each for h-DQN and config 5) of the
# round-4 library, the working tree, nc4 (every forward on 4 column tiles, same lists) and allneed
# (every env in every list: the round-4 work through the round-5 pass structure)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05c
mkdir -p $O
L="tools/variants/lib_r05base.so merging-gym_amd/merging_gym/libmerging_hip.so tools/variants/lib_nc4.so tools/variants/lib_allneed.so"
echo "== ab hdqn" && timeout -k 10 500 python tools/ab_hdqn.py $L --rounds 2 > $O/ab_hdqn.log 2>&1; rc=$?; tail -4 $O/ab_hdqn.log; [ $rc -eq 0 ] || exit $rc
echo "== ab qnet" && timeout -k 10 500 python tools/ab_kernels.py --qnet $L > $O/ab_qnet.log 2>&1; rc=$?; tail -4 $O/ab_qnet.log; exit $rc
