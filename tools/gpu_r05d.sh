# r05d: SQ counters of the policy kernels, round-4 library vs the allneed variant (same forwards
# through the round-5 pass structure) vs the working tree (tools/profile_policy.py workload)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05d
mkdir -p $O
for lib in tools/variants/lib_r05base.so tools/variants/lib_allneed.so merging-gym_amd/merging_gym/libmerging_hip.so; do
  tag=$(basename $lib .so); mkdir -p $O/$tag
  export MERGING_HIP_LIB=$PWD/$lib
  i=0
  for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM" \
             "MfmaUtil SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_BF16" "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_IFETCH" \
             "SQC_ICACHE_HITS SQC_ICACHE_MISSES" "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_WR"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/$tag/p$i -o p -- python tools/profile_policy.py > $O/$tag/p$i.log 2>&1 || echo "$tag pass $i ($set) failed"
  done
  echo "$tag done"
done
