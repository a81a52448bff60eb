# PMC counter passes over the fused dwpw micro-benchmark (tools/gpu/bench_dwpw.py), one rocprofv3 run
# per pass.   bash tools/gpu/pmc_dwpw.sh <outdir> "<B C H W>" <kernel-substring>
cd "$GRAFT_REPO_ROOT"
OUT=$1; SHAPE=$2; KERN=${3:-dwpw_kernel}
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for pass in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
            "TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum" \
            "FETCH_SIZE"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $pass -d "$OUT/p$i" -o run -- python3 -u tools/gpu/bench_dwpw.py $SHAPE \
    > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed $?"; tail -5 "$OUT/p$i.log"; exit 1; }
  db=$(find "$OUT/p$i" -name '*.db' | head -n 1)
  python3 tools/pmc_summary.py "$db" "$KERN"
  python3 tools/pmc_summary.py "$db" "pw_resident_kernel"
done
