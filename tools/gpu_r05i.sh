# r05i: SQ counters of the policy kernels, round-4 library vs the working tree (r05h build), and a
# dump of mg_qnet_forward outputs for the summation-order study (tools/mfma_order_dump.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05i
mkdir -p $O
timeout -k 10 300 python tools/mfma_order_dump.py $O/qdump.npz > $O/dump.log 2>&1 || { echo "dump failed"; tail -3 $O/dump.log; exit 1; }
for lib in tools/variants/lib_r05base.so merging-gym_amd/merging_gym/libmerging_hip.so; do
  tag=$(basename $lib .so); mkdir -p $O/$tag
  export MERGING_HIP_LIB=$PWD/$lib
  i=0
  for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM" \
             "MfmaUtil SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_BF16" "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH VALUBusy" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/$tag/p$i -o p -- python tools/profile_policy.py > $O/$tag/p$i.log 2>&1 || echo "$tag pass $i ($set) failed"
  done
  echo "$tag done"
done
