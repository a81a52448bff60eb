# Round measurement record, part 2 (after tools/gpu/check.sh): rocprofv3 kernel stats of the default
# bench and the PMC HBM-traffic passes of its dominant family; usage on the box:
#   bash tools/gpu/record_prof.sh <outdir> <kernel-substring>
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/r02}
KERN=${2:-conv_x3v2_kernel}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 -u bench.py --no-cpu-baseline > "$OUT/bench_under_rocprof.json" 2> "$OUT/rocprof.err" ||
  { echo "rocprof stats failed $?"; tail -20 "$OUT/rocprof.err"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
  python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-roofline > "$OUT/pmc_fetch.log" 2>&1 ||
  { echo "pmc fetch failed $?"; tail -20 "$OUT/pmc_fetch.log"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
  python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-roofline > "$OUT/pmc_write.log" 2>&1 ||
  { echo "pmc write failed $?"; tail -20 "$OUT/pmc_write.log"; exit 1; }
python3 tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" "$KERN" "$OUT/pmc_traffic.json" config=main
