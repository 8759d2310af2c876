# Round-3 GPU session: h-DQN GPU tests, bench, the 2^22 placement probe, the bench with the 2^22
# env allocated before the legs (with and without the Q-net legs), then the SQ compute-side
# passes (MFMA, LDS). Usage: TAG=r03e bash tools/gpu_r03_probe.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r03e}
O=gpurun_out/$TAG
mkdir -p $O
echo "== pytest hdqn" && { timeout -k 10 600 python -u -m pytest tests/test_gpu_hdqn.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_hdqn.log 2>&1; rc=$?; tail -2 $O/pytest_hdqn.log; [ $rc -eq 0 ]; } \
&& echo "== bench default" && timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 && tail -1 $O/bench_default.log | cut -c1-200 \
&& echo "== placement" && timeout -k 10 300 python tools/placement_probe.py 8 > $O/placement.json 2> $O/placement.err \
&& echo "== bench last prealloc" && timeout -k 10 400 python bench.py --no-cpu-baseline --size2-when last --size2-prealloc > $O/bench_last_prealloc.log 2>&1 \
&& echo "== bench last prealloc noq" && timeout -k 10 400 python bench.py --no-cpu-baseline --size2-when last --size2-prealloc --qnet-launches 0 > $O/bench_last_prealloc_noq.log 2>&1 \
&& echo "== pmc valu" && bash tools/pmc_valu.sh $O/pmcv \
&& echo "== all ok"
