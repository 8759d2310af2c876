# r04h: config-5 A/B of the no-wait statistics (finish_episode_nowait) against the committed build
# and the register-statistics variant; the step kernel's finishing cost at 2^20 (statistics off,
# terminal observations off); config-5 parity tests on the no-wait build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04h
mkdir -p $O
echo "== ab qnet" && MG_AB_FLAGS=1 timeout -k 10 300 python tools/ab_kernels.py tools/variants/lib_r0latphhb.so tools/variants/lib_sreg.so tools/variants/lib_nowait.so --qnet --rounds 5 --warm 1200 > $O/ab_qnet.log 2>&1 && tail -3 $O/ab_qnet.log \
&& echo "== ab step, stats on" && timeout -k 10 200 python tools/ab_kernels.py tools/variants/lib_r0latphhb.so --rounds 5 --warm 1200 > $O/ab_step.log 2>&1 && tail -2 $O/ab_step.log | head -1 \
&& echo "== ab step, stats off" && MG_AB_NOSTATS=1 timeout -k 10 200 python tools/ab_kernels.py tools/variants/lib_r0latphhb.so --rounds 5 --warm 1200 > $O/ab_step_nostats.log 2>&1 && tail -2 $O/ab_step_nostats.log | head -1 \
&& echo "== ab step, stats off, no terminal obs" && MG_AB_NOSTATS=1 MG_AB_NOFOBS=1 timeout -k 10 200 python tools/ab_kernels.py tools/variants/lib_r0latphhb.so --rounds 5 --warm 1200 > $O/ab_step_nofin.log 2>&1 && tail -2 $O/ab_step_nofin.log | head -1 \
&& echo "== pytest qnet" && timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_qnet.py tests/test_gpu_episode_stats.py > $O/pytest_qnet.log 2>&1 && tail -2 $O/pytest_qnet.log \
&& echo "== all ok"
