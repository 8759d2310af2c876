set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
V=merging-gym_amd/variants
for f in 0 1 0 1 0 1; do MG_AB_FLAGS=$f timeout -k 10 200 python tools/ab_kernels.py $V/lib_new.so --qnet --rounds 3 --warm 1200 2>&1 | grep "lib_" | sed "s/^/flags=$f /" || exit 1; done
