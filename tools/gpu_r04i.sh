# r04i: the no-wait statistics in every batched kernel (lib_nowait2 = the working tree) against the
# committed build (lib_r0latphhb): step / rollout, config-5, h-DQN A/Bs; then the GPU test suite,
# smoke and a default bench on the working tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04i
mkdir -p $O
V="tools/variants/lib_r0latphhb.so tools/variants/lib_nowait2.so"
echo "== ab step/rollout" && timeout -k 10 300 python tools/ab_kernels.py $V --rounds 7 --warm 1200 > $O/ab_step.log 2>&1 && tail -3 $O/ab_step.log | head -2 \
&& echo "== ab qnet" && MG_AB_FLAGS=1 timeout -k 10 300 python tools/ab_kernels.py $V --qnet --rounds 5 --warm 1200 > $O/ab_qnet.log 2>&1 && tail -2 $O/ab_qnet.log \
&& echo "== ab hdqn" && timeout -k 10 400 python tools/ab_hdqn.py $V > $O/ab_hdqn.log 2>&1 && tail -3 $O/ab_hdqn.log \
&& echo "== pytest gpu" && timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 && tail -2 $O/pytest_gpu.log \
&& echo "== smoke" && timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 && tail -1 $O/smoke.log \
&& echo "== bench" && timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 && tail -1 $O/bench_default.log | cut -c1-300 \
&& echo "== size2 probe2" && timeout -k 10 200 python tools/size2_probe2.py > $O/size2_probe2.txt 2>&1 && cat $O/size2_probe2.txt \
&& echo "== all ok"
