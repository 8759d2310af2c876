#!/bin/bash
# r04ac: non-temporal env-state loads (load_env) against the product, step kernel, both orders
set -o pipefail
O=gpurun_out/r04ac
mkdir -p $O
echo "== ab step" && MG_AB_FLAGS=1 timeout -k 10 400 python tools/ab_kernels.py tools/variants/lib_sc.so tools/variants/lib_ntload.so --rounds 10 --warm 1200 --rollouts 2 > $O/ab_step.log 2>&1 && tail -3 $O/ab_step.log | head -2 \
&& echo "== ab step rev" && MG_AB_FLAGS=1 timeout -k 10 400 python tools/ab_kernels.py tools/variants/lib_ntload.so tools/variants/lib_sc.so --rounds 10 --warm 1200 --rollouts 2 > $O/ab_step_rev.log 2>&1 && tail -3 $O/ab_step_rev.log | head -2 \
&& echo "== ab step 2^22" && MG_AB_FLAGS=1 timeout -k 10 400 python tools/ab_kernels.py tools/variants/lib_sc.so tools/variants/lib_ntload.so --envs 4194304 --rounds 6 --warm 600 --rollouts 1 > $O/ab_step22.log 2>&1 && tail -3 $O/ab_step22.log | head -2 \
&& echo "== ab replay" && MG_AB_FLAGS=1 timeout -k 10 400 python tools/ab_kernels.py tools/variants/lib_sc.so tools/variants/lib_ntload2.so --replay --rounds 8 > $O/ab_replay.log 2>&1 && tail -3 $O/ab_replay.log \
&& echo "== ab replay rev" && MG_AB_FLAGS=1 timeout -k 10 400 python tools/ab_kernels.py tools/variants/lib_ntload2.so tools/variants/lib_sc.so --replay --rounds 8 > $O/ab_replay_rev.log 2>&1 && tail -3 $O/ab_replay_rev.log \
&& echo "== all ok"
