# r05y: h-DQN phase clocks: committed source (opponent meta compacted) vs the lower passes compacted with env-wave tails
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05y
mkdir -p $O
timeout -k 10 300 python tools/clk_probe.py tools/variants/lib_clk_hhead.so tools/variants/lib_clk_hlow.so > $O/clk.log 2>&1; rc=$?; grep -v amdgpu.ids $O/clk.log | tail -14; exit $rc
