# r04g: config-5 A/B (statistics in registers; statistics ablation), int32 / VALU PMC passes for the
# round-3-equivalent library and the current one, and a driver-style bench (2^22 windows without
# the idle gap).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04g
mkdir -p $O
echo "== ab qnet" && MG_AB_FLAGS=1 timeout -k 10 300 python tools/ab_kernels.py tools/variants/lib_base.so tools/variants/lib_r0latphhb.so tools/variants/lib_sreg.so --qnet --rounds 5 --warm 1200 > $O/ab_qnet.log 2>&1 && tail -3 $O/ab_qnet.log \
&& echo "== ab qnet, no statistics" && MG_AB_FLAGS=1 MG_AB_NOSTATS=1 timeout -k 10 300 python tools/ab_kernels.py tools/variants/lib_r0latphhb.so --qnet --rounds 5 --warm 1200 > $O/ab_qnet_nostats.log 2>&1 && tail -1 $O/ab_qnet_nostats.log \
&& for lib in base r0latphhb; do for pass in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F32"; do \
     tag=$(echo $pass | cut -c10-20 | tr ' ' '_'); echo "== pmc $lib $tag"; \
     MERGING_HIP_LIB=$PWD/tools/variants/lib_$lib.so timeout -s KILL 150 rocprofv3 --pmc $pass --output-format csv -d $O/pmc_$lib/$tag -o p -- python tools/profile_valu.py > $O/pmc_${lib}_$tag.log 2>&1 || exit 1; done; done \
&& echo "== bench driver-style" && timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20.log 2>&1 && tail -1 $O/bench_k20.log | cut -c1-200 \
&& echo "== all ok"
