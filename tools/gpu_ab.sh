# A/B kernel variants in one process (interleaved rounds, same GPU).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
V=merging-gym_amd/variants
echo "== ab 2^20 T16" && timeout -k 10 300 python tools/ab_kernels.py $V/lib_*.so --rounds 6 > gpurun_out/ab1.log 2>&1; rc=$?; tail -6 gpurun_out/ab1.log | cut -c1-230; [ $rc -eq 0 ] \
&& echo "== ab 2^20 T64" && timeout -k 10 300 python tools/ab_kernels.py $V/lib_nt.so $V/lib_sc1all.so --T 64 --rollouts 2 --rounds 4 > gpurun_out/ab3.log 2>&1 && tail -3 gpurun_out/ab3.log | cut -c1-230 \
&& echo "== ab 2^22" && timeout -k 10 300 python tools/ab_kernels.py $V/lib_nt.so $V/lib_sc1all.so $V/lib_sc1out.so --envs 4194304 --rounds 4 > gpurun_out/ab2.log 2>&1 && tail -4 gpurun_out/ab2.log | cut -c1-230
