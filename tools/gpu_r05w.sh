# r05w: h-DQN timing probe -- the lower (and meta) passes at three column tiles (timing only; the
# fourth tile's choices are not computed in the variants)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05w
mkdir -p $O
echo "== ab hdqn" && timeout -k 10 600 python tools/ab_hdqn.py tools/variants/lib_r05base.so merging-gym_amd/merging_gym/libmerging_hip.so tools/variants/lib_hd_low3.so tools/variants/lib_hd_all3.so --rounds 4 > $O/ab_hdqn.log 2>&1; rc=$?; tail -4 $O/ab_hdqn.log; exit $rc
