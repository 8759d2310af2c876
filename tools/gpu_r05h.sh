# r05h: scatter entries read ahead of the forward; h-DQN A/B incl. ga2 (L2 fragment ring 2 deep: the
# OPP 3 instance spills 10 VGPRs at 3); config-5 A/B; the MFMA summation-order probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05h
mkdir -p $O
echo "== probe" && timeout -k 10 300 python tools/mfma_order_probe.py > $O/probe.log 2>&1; rc=$?; cat $O/probe.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
echo "== ab hdqn" && timeout -k 10 400 python tools/ab_hdqn.py tools/variants/lib_r05base.so merging-gym_amd/merging_gym/libmerging_hip.so tools/variants/lib_ga2.so --rounds 3 > $O/ab_hdqn.log 2>&1; rc=$?; tail -3 $O/ab_hdqn.log; [ $rc -eq 0 ] || exit $rc
echo "== ab qnet" && timeout -k 10 400 python tools/ab_kernels.py --qnet tools/variants/lib_r05base.so merging-gym_amd/merging_gym/libmerging_hip.so > $O/ab_qnet.log 2>&1; rc=$?; tail -2 $O/ab_qnet.log; exit $rc
