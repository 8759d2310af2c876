# r04o: replay store ablations (obs reads reduced to one 8-byte load per row; row stores skipped)
# against the product build; the statistics-clear test.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04o
mkdir -p $O
echo "== pytest clear" && timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_episode_stats.py > $O/pytest_stats.log 2>&1 && tail -2 $O/pytest_stats.log \
&& echo "== ab replay" && timeout -k 10 300 python tools/ab_kernels.py tools/variants/lib_rp_base.so tools/variants/lib_rp_noobs.so tools/variants/lib_rp_nostore.so --replay --rounds 8 > $O/ab_replay.log 2>&1 && tail -3 $O/ab_replay.log \
&& echo "== all ok"
