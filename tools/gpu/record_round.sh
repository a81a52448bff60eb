# Round measurement record: GPU tests (+ exact parity counts), PMC HBM traffic of the dominant family,
# the default bench line (roofline.traffic from that PMC run, per-layer table), rocprofv3 kernel stats
# of the same bench command, and the reduced-precision synthesis line.  usage on the box:
#   bash tools/gpu/record_round.sh <outdir> [kernel-family]
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/record}
KERN=${2:-conv_x4_kernel}
mkdir -p "$OUT"
export TMPDIR=/tmp
# (no -x: a failing test is recorded with the rest of the suite and the measurements still run;
# a time limit, abort or crash ends the record)
MLIC_PARITY_OUT="$OUT/parity_counts.json" timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 \
  --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; grep -E "^FAILED|^E  " "$OUT/gpu_tests.log" | head -20; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
tail -1 "$OUT/gpu_tests.log"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
  python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-roofline > "$OUT/pmc_fetch.log" 2>&1 ||
  { echo "pmc fetch failed $?"; tail -20 "$OUT/pmc_fetch.log"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
  python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-roofline > "$OUT/pmc_write.log" 2>&1 ||
  { echo "pmc write failed $?"; tail -20 "$OUT/pmc_write.log"; exit 1; }
python3 tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" "$KERN" "$OUT/traffic.json" config=main || exit 1
timeout -k 10 600 python3 -u bench.py --traffic-json "$OUT/traffic.json" --layers-out "$OUT/layers.tsv" \
  > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed $?"; tail -30 "$OUT/bench.err"; exit 1; }
head -c 300 "$OUT/bench.json"; echo
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 -u bench.py --no-cpu-baseline --traffic-json "$OUT/traffic.json" > "$OUT/bench_under_rocprof.json" \
  2> "$OUT/rocprof.err" || { echo "rocprof stats failed $?"; tail -20 "$OUT/rocprof.err"; exit 1; }
rm -f "$OUT"/prof/run_kernel_trace.csv
# the timed workload alone (no profiled passes): its per-launch averages are the ones the line's
# roofline divides by (the run above also holds the one-lane isolated pass, whose launches are shorter)
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_timed" -o run -- \
  python3 -u bench.py --no-cpu-baseline --no-roofline > "$OUT/bench_under_rocprof_timed.json" \
  2> "$OUT/rocprof_timed.err" || { echo "rocprof timed stats failed $?"; tail -20 "$OUT/rocprof_timed.err"; exit 1; }
rm -f "$OUT"/prof_timed/run_kernel_trace.csv
timeout -k 10 400 python3 -u bench.py --synth-fp16 --no-cpu-baseline --traffic-json "$OUT/traffic.json" \
  --layers-out "$OUT/layers_synth_fp16.tsv" > "$OUT/bench_synth_fp16.json" 2> "$OUT/bench_synth_fp16.err" ||
  { echo "bench synth-fp16 failed $?"; tail -20 "$OUT/bench_synth_fp16.err"; exit 1; }
head -c 300 "$OUT/bench_synth_fp16.json"; echo
