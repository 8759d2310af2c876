# r05s: phase clocks of the config-5 kernel: round-4 source, round-5 HEAD, the net-split other-net path
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05s
mkdir -p $O
timeout -k 10 300 python tools/clk_probe_qnet.py tools/variants/lib_clk_q5base.so tools/variants/lib_clk_q5head.so tools/variants/lib_clk_q5split.so > $O/clk.log 2>&1; rc=$?; grep -v amdgpu.ids $O/clk.log | tail -24; exit $rc
