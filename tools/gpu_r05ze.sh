# r05ze: h-DQN Q-net waves' phase segments on the kernel with the bytes and inputs read ahead (tools/clk_segments.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05ze
mkdir -p $O
timeout -k 10 300 python tools/clk_segments.py tools/variants/lib_clk_hnow2.so > $O/seg.log 2>&1; rc=$?; grep -v amdgpu.ids $O/seg.log | tail -6; exit $rc
