# SQ compute-side counters of the four hot kernels (tools/profile_valu.py), one pass per group:
# VALU / SALU issue, instruction mix, wave time split, MFMA pipe (MfmaUtil = rocprofv3's derived
# SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x SIMDs)) and LDS bank conflicts.
# Usage (GPU box): bash tools/pmc_valu.sh OUTDIR
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${1:-gpurun_out/pmcv}
mkdir -p $O
i=0
for set in "VALUBusy SALUBusy" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64" \
           "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F32" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" \
           "MfmaUtil SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_COEXEC_CYCLES" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o p -- python tools/profile_valu.py > $O/p$i.log 2>&1 || { echo "pass $i ($set) failed"; tail -5 $O/p$i.log; exit 1; }
  echo "pass $i ok"
done
