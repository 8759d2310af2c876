# Round-3 GPU session: smoke -> GPU tests -> driver-style bench -> full bench -> rocprof kernel
# stats [-> PMC passes]. Every GPU step has its own time limit and the chain stops at the first
# failure. Usage: TAG=r03b bash tools/gpu_r03.sh [pmc]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r03}
O=gpurun_out/$TAG
mkdir -p $O
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log \
&& echo "== pytest gpu" && { timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ]; } \
&& echo "== bench driver-style" && timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20.log 2>&1 && tail -1 $O/bench_k20.log | cut -c1-400 \
&& echo "== bench default" && timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 && tail -1 $O/bench_default.log | cut -c1-300 \
&& echo "== rocprof stats" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o $TAG -- python bench.py --steps 300 --warmup 20 --no-cpu-baseline --size2-envs 0 > $O/prof.log 2>&1 && tail -1 $O/prof.log | cut -c1-200 \
&& if [ "$1" = "pmc" ]; then
  echo "== pmc fetch" && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python tools/profile_pmc.py > $O/pmc_fetch.log 2>&1 \
  && echo "== pmc write" && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python tools/profile_pmc.py > $O/pmc_write.log 2>&1
fi \
&& echo "== all ok"
