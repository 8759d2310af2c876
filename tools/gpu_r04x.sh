# r04x: LLVM AMDGPU scheduler strategies (-mllvm -amdgpu-sched-strategy=...) for the whole library,
# in-process A/B on every leg against the product build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04x
mkdir -p $O
V="tools/variants/lib_rp_base.so tools/variants/lib_sched_max-ilp.so tools/variants/lib_sched_max-memory-clause.so tools/variants/lib_sched_iterative-ilp.so"
echo "== ab step/rollout" && MG_AB_FLAGS=1 timeout -k 10 400 python tools/ab_kernels.py $V --rounds 6 --warm 1200 > $O/ab_step.log 2>&1 && tail -5 $O/ab_step.log | head -4 \
&& echo "== ab qnet" && MG_AB_FLAGS=1 timeout -k 10 400 python tools/ab_kernels.py $V --qnet --rounds 4 --warm 1200 > $O/ab_qnet.log 2>&1 && tail -4 $O/ab_qnet.log \
&& echo "== ab hdqn" && timeout -k 10 500 python tools/ab_hdqn.py $V > $O/ab_hdqn.log 2>&1 && tail -4 $O/ab_hdqn.log \
&& echo "== all ok"
