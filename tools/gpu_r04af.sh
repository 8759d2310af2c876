# r04af: the end-of-session confirmation pass (product unchanged since r04aa): smoke, GPU suite, bench (default and driver-style k20),
# rocprofv3 kernel stats of the bench, HBM traffic (FETCH_SIZE / WRITE_SIZE passes)
# and a 2-rank gloo rehearsal on the one GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04af
mkdir -p $O
echo "== smoke" && timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 && tail -1 $O/smoke.log \
&& echo "== pytest gpu" && timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 && tail -2 $O/pytest_gpu.log \
&& echo "== bench default" && timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 && tail -1 $O/bench_default.log | cut -c1-200 \
&& echo "== bench k20" && timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20.log 2>&1 && tail -1 $O/bench_k20.log | cut -c1-200 \
&& echo "== rocprof stats" && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o r04af -- python bench.py --steps 300 --warmup 20 --no-cpu-baseline > $O/prof.log 2>&1 && tail -1 $O/prof.log | cut -c1-200 \
&& echo "== pmc fetch" && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python tools/profile_pmc.py > $O/pmc_fetch.log 2>&1 \
&& echo "== pmc write" && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python tools/profile_pmc.py > $O/pmc_write.log 2>&1 \
&& echo "== 2-rank rehearsal (gloo, shared GPU)" && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 100 --warmup 10 --envs 262144 --dist-backend gloo --rollout-launches 5 > $O/bench_2rank.log 2>&1 && tail -1 $O/bench_2rank.log | cut -c1-300 \
&& echo "== all ok"
