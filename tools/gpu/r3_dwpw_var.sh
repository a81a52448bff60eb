# fused dwpw variant timings (base + tools/gpu/var/libmlic_<v>.so) and one PMC pass per variant.
#   bash tools/gpu/r3_dwpw_var.sh <outdir> "<variants>" ["<B C H W>"]
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/dwpw_var}; VARS=${2:-base}; SHP=${3:-8 192 544 960}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in $VARS; do
  if [ $v = base ]; then L=mlic_amd/libmlic_hip.so; else L=tools/gpu/var/libmlic_$v.so; fi
  MLIC_HIP_LIB=$PWD/$L timeout -k 10 120 python -u tools/gpu/bench_dwpw.py $SHP > "$OUT/b.tmp" 2>&1 || { echo "bench $v failed"; cat "$OUT/b.tmp"; exit 1; }
  echo "$v $(grep fused "$OUT/b.tmp")" | tee -a "$OUT/var.log"
done
for v in $VARS; do
  if [ $v = base ]; then L=mlic_amd/libmlic_hip.so; else L=tools/gpu/var/libmlic_$v.so; fi
  MLIC_HIP_LIB=$PWD/$L timeout -s KILL 90 rocprofv3 --pmc TA_TA_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum GRBM_GUI_ACTIVE -d "$OUT/pmc_$v" -o run -- python3 -u tools/gpu/bench_dwpw.py $SHP > "$OUT/pmc_$v.log" 2>&1 || { echo "pmc $v failed"; tail -5 "$OUT/pmc_$v.log"; exit 1; }
  echo "== $v"; python3 tools/pmc_summary.py "$(find "$OUT/pmc_$v" -name '*.db' | head -n 1)" dwpw
done
