# A/B kernel variants in one process (interleaved rounds, same GPU).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
V=merging-gym_amd/variants
true \
&& echo "== ab step/rollout 2^20" && timeout -k 10 300 python tools/ab_kernels.py $V/lib_*.so --rounds 12 --warm 1000 > gpurun_out/ab1.log 2>&1 && tail -6 gpurun_out/ab1.log | cut -c1-230
