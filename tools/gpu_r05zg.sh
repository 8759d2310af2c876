# r05zg: round-5 final pass, part 1 (config-5 net split + env-wave tails, h-DQN opponent meta compacted): smoke, the GPU suite, bench (default and driver-style k20), and the
# rocprofv3 kernel statistics of the bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05zg
mkdir -p $O
echo "== smoke" && timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 && tail -1 $O/smoke.log \
&& echo "== pytest gpu" && timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 && tail -2 $O/pytest_gpu.log \
&& echo "== bench k20" && timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20.log 2>&1 && tail -1 $O/bench_k20.log | cut -c1-300 \
&& echo "== bench default" && timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 && tail -1 $O/bench_default.log | cut -c1-300 \
&& echo "== rocprof stats" && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o r05zg -- python bench.py --steps 300 --warmup 20 --no-cpu-baseline > $O/prof.log 2>&1 && tail -1 $O/prof.log | cut -c1-200 \
&& echo "== all ok"
