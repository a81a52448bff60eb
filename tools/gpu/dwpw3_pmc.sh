# PMC passes over the dwpw3 GELU launch (8 x 192 x 544 x 960): issue / wait / busy counters, one pass each
#   bash tools/gpu/dwpw3_pmc.sh <outdir>
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/d3pmc}
mkdir -p "$OUT"
export DWPW_EPI=1 MLIC_DWPW2=${D2FORM:-2}
cd /tmp && export TMPDIR=/tmp
run() {  # name counters...
  local n=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d "$GRAFT_REPO_ROOT/$OUT/$n" -o pmc --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/tools/gpu/dwpw_ab.py" v3 > "$GRAFT_REPO_ROOT/$OUT/$n.log" 2>&1 || { echo "pass $n failed"; tail -5 "$GRAFT_REPO_ROOT/$OUT/$n.log"; exit 1; }
}
run a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES
run b SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS
run c SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
echo pmc done
