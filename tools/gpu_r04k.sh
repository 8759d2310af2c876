# r04k: the no-wait statistics kept in the Q-net kernels only (lib_nowait3 = the working tree):
# A/B against the committed build on every leg; the clear transient at 2^20; GPU suite + bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04k
mkdir -p $O
V="tools/variants/lib_r0latphhb.so tools/variants/lib_nowait3.so"
echo "== ab qnet" && MG_AB_FLAGS=1 timeout -k 10 300 python tools/ab_kernels.py $V --qnet --rounds 6 --warm 1200 > $O/ab_qnet.log 2>&1 && tail -2 $O/ab_qnet.log \
&& echo "== ab step/rollout" && timeout -k 10 400 python tools/ab_kernels.py $V --rounds 10 --warm 1200 > $O/ab_step.log 2>&1 && tail -3 $O/ab_step.log | head -2 \
&& echo "== size2 probe2 at 2^20" && timeout -k 10 200 python tools/size2_probe2.py 1048576 > $O/probe2_2p20.txt 2>&1 && cat $O/probe2_2p20.txt \
&& echo "== pytest gpu" && timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 && tail -2 $O/pytest_gpu.log \
&& echo "== bench k20" && timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20.log 2>&1 && tail -1 $O/bench_k20.log | cut -c1-200 \
&& echo "== bench default" && timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 && tail -1 $O/bench_default.log | cut -c1-200 \
&& echo "== all ok"
