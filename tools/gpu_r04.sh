# Round-4 GPU pass: smoke -> all GPU tests -> default bench -> driver-style bench -> rocprof stats.
# Every GPU step has its own time limit; the chain stops at the first failure.
# Usage: TAG=r04a bash tools/gpu_r04.sh   (SKIP_TESTS=1 / SKIP_PROF=1 to drop a step)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r04}
O=gpurun_out/$TAG
mkdir -p $O
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log \
&& { [ -n "$SKIP_TESTS" ] || { echo "== pytest gpu" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ]; }; } \
&& echo "== bench default" && timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 && tail -1 $O/bench_default.log | cut -c1-300 \
&& echo "== bench driver-style" && timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20.log 2>&1 && tail -1 $O/bench_k20.log | cut -c1-200 \
&& { [ -n "$SKIP_PROF" ] || { echo "== rocprof stats" && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o $TAG -- python bench.py --no-cpu-baseline > $O/prof.log 2>&1 && tail -1 $O/prof.log | cut -c1-200; }; } \
&& echo "== all ok"
