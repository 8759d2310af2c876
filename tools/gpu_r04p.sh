# r04p: the replay store with every per-step load issued before the chunk's first barrier
# (lib_rp_pre = the working tree; rp_pre4: 4 steps per write block) against the product build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04p
mkdir -p $O
echo "== pytest replay" && timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_replay.py > $O/pytest_replay.log 2>&1 && tail -2 $O/pytest_replay.log \
&& echo "== ab replay" && timeout -k 10 300 python tools/ab_kernels.py tools/variants/lib_rp_base.so tools/variants/lib_rp_pre.so tools/variants/lib_rp_pre4.so --replay --rounds 8 > $O/ab_replay.log 2>&1 && tail -3 $O/ab_replay.log \
&& echo "== all ok"
