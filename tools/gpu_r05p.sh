# r05p: config-5 A/B, round-4 vs round-5 library, 10 rounds, twice (box variance check)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05p
mkdir -p $O
for i in 1 2; do
  timeout -k 10 500 python tools/ab_kernels.py --qnet tools/variants/lib_r05base.so merging-gym_amd/merging_gym/libmerging_hip.so --rounds 10 > $O/ab_qnet_$i.log 2>&1 || exit 1
  tail -2 $O/ab_qnet_$i.log
done
timeout -k 10 400 python tools/ab_hdqn.py tools/variants/lib_r05base.so merging-gym_amd/merging_gym/libmerging_hip.so --rounds 3 > $O/ab_hdqn.log 2>&1; tail -2 $O/ab_hdqn.log
