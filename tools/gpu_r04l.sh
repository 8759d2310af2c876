# r04l: the no-wait statistics in the one-step kernel past the Infinity Cache (2^22 envs), where the
# finishing lanes' read-modify-write misses to DRAM: lib_nowait2 (step + rollout no-wait) against the
# committed round-3 paths; then the reduction timing with events right around its launches.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04l
mkdir -p $O
V="tools/variants/lib_r0latphhb.so tools/variants/lib_nowait2.so"
echo "== ab step/rollout 2^22" && timeout -k 10 400 python tools/ab_kernels.py $V --envs 4194304 --rounds 6 --warm 1500 --rollouts 2 > $O/ab_step_2p22.log 2>&1 && tail -3 $O/ab_step_2p22.log | head -2 \
&& echo "== ab step/rollout 2^22 reversed" && timeout -k 10 400 python tools/ab_kernels.py tools/variants/lib_nowait2.so tools/variants/lib_r0latphhb.so --envs 4194304 --rounds 6 --warm 1500 --rollouts 2 > $O/ab_step_2p22_rev.log 2>&1 && tail -3 $O/ab_step_2p22_rev.log | head -2 \
&& echo "== bench k20" && timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20.log 2>&1 && tail -1 $O/bench_k20.log | cut -c1-200 \
&& echo "== pytest full-size policy" && timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_qnet.py tests/test_gpu_hdqn.py -k full_size > $O/pytest_full.log 2>&1 && tail -2 $O/pytest_full.log \
&& echo "== all ok"
