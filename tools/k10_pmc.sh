# PMC passes over the K10 'down' and 'qkv' GEMMs alone (tools/pmc.sh per GEMM)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
export PMC_SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS;SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS;TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE;FETCH_SIZE"
for g in down qkv; do
  K10_ONLY=$g K10_E5=0 bash tools/pmc.sh k10_$g linear_f16x3 -- python3 tools/k10_probe.py || exit 1
done
