# Quick GPU check: smoke -> all GPU tests -> default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== smoke" && timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log \
&& echo "== pytest gpu" && { timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ]; } \
&& echo "== bench" && timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log | cut -c1-1500
