# Round measurement record, part 2: one bench line per BASELINE config workload, plus the 8-rank
# emulations (rank 0's job share on one GPU with 1/8 of the host cores); usage on the box:
#   bash tools/gpu/record_configs.sh <outdir>
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/configs}
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in ${CONFIGS-kodak s1080 sd1080 vbr-mixed kodak-sweep}; do
  timeout -k 10 400 python3 -u bench.py --config "$c" --records-out "$OUT/records_$c.json" > "$OUT/bench_$c.json" \
    2> "$OUT/bench_$c.err" || { echo "bench $c failed $?"; tail -20 "$OUT/bench_$c.err"; exit 1; }
  echo "$c: $(head -c 300 "$OUT/bench_$c.json")"
done
for c in ${EMU-main kodak-sweep vbr-mixed}; do
  timeout -k 10 400 python3 -u bench.py --config "$c" --emulate-world 8 --emulate-rank 0 --no-cpu-baseline \
    > "$OUT/bench_${c}_emu8r0.json" 2> "$OUT/bench_${c}_emu8r0.err" ||
    { echo "emu $c failed $?"; tail -20 "$OUT/bench_${c}_emu8r0.err"; exit 1; }
  echo "$c emu8r0: $(head -c 300 "$OUT/bench_${c}_emu8r0.json")"
done
