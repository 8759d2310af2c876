# r05zi: h-DQN phase segments: committed kernel vs the lower passes listed by the env waves (r05zh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05zi
mkdir -p $O
timeout -k 10 200 python tools/clk_segments.py tools/variants/lib_clk_hnow3.so > $O/seg_head.log 2>&1 && timeout -k 10 200 python tools/clk_segments.py tools/variants/lib_clk_hlist.so > $O/seg_list.log 2>&1; rc=$?; grep -v amdgpu.ids $O/seg_head.log | tail -3; grep -v amdgpu.ids $O/seg_list.log | tail -3; exit $rc
