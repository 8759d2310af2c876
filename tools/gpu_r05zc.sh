# r05zc: h-DQN Q-net waves' phase segments on the kept round-5 kernel (tools/clk_segments.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05zc
mkdir -p $O
timeout -k 10 300 python tools/clk_segments.py tools/variants/lib_clk_hnow.so > $O/seg.log 2>&1; rc=$?; grep -v amdgpu.ids $O/seg.log | tail -6; exit $rc
