# r05q: phase clocks of the config-5 kernel, round-4 source vs the working tree (tools/clk_variant.py q5base / q5)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05q
mkdir -p $O
timeout -k 10 300 python tools/clk_probe_qnet.py tools/variants/lib_clk_q5base.so tools/variants/lib_clk_q5new.so > $O/clk.log 2>&1; rc=$?; grep -v amdgpu.ids $O/clk.log | tail -12; exit $rc
