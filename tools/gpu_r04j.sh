# r04j: the statistics clear as one full-record pass (size2_probe2), and a longer step / rollout
# A/B of the no-wait statistics (the r04i rollout medians were noisy).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04j
mkdir -p $O
V="tools/variants/lib_r0latphhb.so tools/variants/lib_nowait2.so"
echo "== size2 probe2" && timeout -k 10 200 python tools/size2_probe2.py > $O/size2_probe2.txt 2>&1 && cat $O/size2_probe2.txt \
&& echo "== ab step/rollout" && timeout -k 10 400 python tools/ab_kernels.py $V --rounds 12 --warm 1200 > $O/ab_step.log 2>&1 && tail -3 $O/ab_step.log | head -2 \
&& echo "== ab step/rollout, reversed order" && timeout -k 10 400 python tools/ab_kernels.py tools/variants/lib_nowait2.so tools/variants/lib_r0latphhb.so --rounds 12 --warm 1200 > $O/ab_step_rev.log 2>&1 && tail -3 $O/ab_step_rev.log | head -2 \
&& echo "== bench k20" && timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20.log 2>&1 && tail -1 $O/bench_k20.log | cut -c1-200 \
&& echo "== all ok"
