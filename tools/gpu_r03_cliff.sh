# Round-3 GPU session: counter list, parity subset, bench (2^22 leg first), then the 2^22 leg after
# every other leg (the r02d cliff) with its env allocated late and early. Usage: TAG=r03c bash tools/gpu_r03_cliff.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r03c}
O=gpurun_out/$TAG
mkdir -p $O
echo "== counters" && { timeout -k 10 120 rocprofv3 -L > $O/avail.txt 2>&1 || timeout -k 10 120 rocprofv3 --list-avail > $O/avail.txt 2>&1; grep -ciE "mfma|utcl|tlb" $O/avail.txt; true; } \
&& echo "== pytest subset" && { timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_episode_stats.py tests/test_dropin.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ]; } \
&& echo "== bench default" && timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 && tail -1 $O/bench_default.log | cut -c1-200 \
&& echo "== bench size2 last" && timeout -k 10 400 python bench.py --no-cpu-baseline --size2-when last > $O/bench_size2_last.log 2>&1 && tail -1 $O/bench_size2_last.log | cut -c1-120 \
&& echo "== bench size2 last prealloc" && timeout -k 10 400 python bench.py --no-cpu-baseline --size2-when last --size2-prealloc > $O/bench_size2_last_prealloc.log 2>&1 && tail -1 $O/bench_size2_last_prealloc.log | cut -c1-120 \
&& echo "== all ok"
