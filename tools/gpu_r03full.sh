# Full GPU pass: smoke -> all GPU tests -> Q-net A/B (tools/variants) -> default bench -> driver-style
# bench. Every GPU step has its own time limit; the chain stops at the first failure.
# Usage: TAG=r03ag bash tools/gpu_r03full.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r03full}
O=gpurun_out/$TAG
mkdir -p $O
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log \
&& echo "== pytest gpu" && { timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ]; } \
&& echo "== ab qnet" && timeout -k 10 300 python tools/ab_kernels.py tools/variants/lib_*.so --qnet --rounds 5 --warm 1200 > $O/ab_qnet.log 2>&1 && tail -3 $O/ab_qnet.log \
&& echo "== bench default" && timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 && tail -1 $O/bench_default.log | cut -c1-200 \
&& echo "== bench driver-style" && timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20.log 2>&1 && tail -1 $O/bench_k20.log | cut -c1-200 \
&& echo "== all ok"
