# r05k: phase clocks of the h-DQN kernel, round-4 source vs the working tree (tools/clk_variant.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05k
mkdir -p $O
timeout -k 10 300 python tools/clk_probe.py tools/variants/lib_clk_base.so tools/variants/lib_clk_new.so > $O/clk.log 2>&1; rc=$?; grep -v amdgpu.ids $O/clk.log | tail -8; exit $rc
