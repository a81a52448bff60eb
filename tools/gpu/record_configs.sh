# Round measurement record, part 3: one bench line per BASELINE config workload; usage on the box:
#   bash tools/gpu/record_configs.sh <outdir>
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/r02}
mkdir -p "$OUT"
for c in ${CONFIGS:-kodak s1080 sd1080 vbr-mixed kodak-sweep}; do
  timeout -k 10 400 python3 -u bench.py --config "$c" --records-out "$OUT/records_$c.json" > "$OUT/bench_$c.json" \
    2> "$OUT/bench_$c.err" || { echo "bench $c failed $?"; tail -20 "$OUT/bench_$c.err"; exit 1; }
  echo "$c: $(head -c 300 "$OUT/bench_$c.json")"
done
