# kernel time + PMC passes of the packed LocalContext attention; usage: bash tools/gpu/pmc_attn.sh <outdir>
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/pmc_attn}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 -u tools/gpu/attn_packed_bench.py 8 > "$OUT/kt.log" 2>&1 || { echo "kt failed"; tail -5 "$OUT/kt.log"; exit 1; }
grep -h "attn" "$OUT"/kt/run_kernel_stats.csv | cut -c1-200
i=0
for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $pass -d "$OUT/p$i" -o run -- python3 -u tools/gpu/attn_packed_bench.py 8 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  db=$(find "$OUT/p$i" -name '*.db' | head -n 1)
  python3 tools/pmc_summary.py "$db" attn
done
