set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== smoke" && timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -3 gpurun_out/smoke.log \
&& echo "== pytest gpu" && timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -30 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] \
&& echo "== bench" && timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 && tail -2 gpurun_out/bench.log \
&& echo "== rocprof" && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o r01 -- python bench.py --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/prof.log 2>&1 && tail -2 gpurun_out/prof.log
