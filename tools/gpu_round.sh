# One GPU session: smoke -> GPU tests -> bench -> rocprof kernel stats -> PMC passes -> 2-rank rehearsal.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
echo "== smoke" && timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log \
&& echo "== pytest gpu" && { timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ]; } \
&& echo "== bench" && timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log \
&& echo "== rocprof stats" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o $TAG -- python bench.py --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/prof.log 2>&1 && tail -1 gpurun_out/prof.log \
&& echo "== pmc fetch" && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o pmc -- python tools/profile_pmc.py > gpurun_out/pmc_fetch.log 2>&1 \
&& echo "== pmc write" && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o pmc -- python tools/profile_pmc.py > gpurun_out/pmc_write.log 2>&1 \
&& echo "== bench 2^22" && timeout -k 10 300 python bench.py --envs 4194304 --steps 300 --no-cpu-baseline > gpurun_out/bench_4m.log 2>&1 && tail -1 gpurun_out/bench_4m.log | cut -c1-400 \
&& echo "== 2-rank rehearsal (gloo, shared GPU)" && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 100 --warmup 10 --envs 262144 --dist-backend gloo --rollout-launches 5 > gpurun_out/bench_2rank.log 2>&1 && tail -1 gpurun_out/bench_2rank.log | cut -c1-600 \
&& echo "== pmc qnet" && bash tools/pmc_qnet.sh
