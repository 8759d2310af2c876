# A/B of the env kernels' block size (MG_BLOCK = 256 default, 128, 512), in one process,
# interleaved rounds, at 2^20 and 2^22 envs. Variants are built beforehand on the CPU host.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
V=merging-gym_amd/variants
timeout -k 10 300 python -u tools/ab_kernels.py $V/lib_b256.so $V/lib_b128.so $V/lib_b512.so --rounds 10 --warm 1000 > gpurun_out/ab_blk20.log 2>&1 && tail -8 gpurun_out/ab_blk20.log | cut -c1-250 \
&& timeout -k 10 300 python -u tools/ab_kernels.py $V/lib_b256.so $V/lib_b128.so $V/lib_b512.so --envs 4194304 --rounds 6 --warm 1000 > gpurun_out/ab_blk22.log 2>&1 && tail -8 gpurun_out/ab_blk22.log | cut -c1-250
