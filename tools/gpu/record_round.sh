# Round measurement record.  usage on the box:
#   bash tools/gpu/record_round.sh <outdir> [kernel-family] [stages]
# stages (default "tests pmc bench decode rocprof"):
#   tests    GPU suite (workspace + outputs NaN-poisoned, tests/conftest.py) with exact parity counts
#   pmc      FETCH_SIZE / WRITE_SIZE of the dominant family over the isolated pass's launches
#            (one lane, 8 images: bench.py --lanes 1 --batch 8 --split 1), tools/pmc_traffic.py -> traffic.json
#   bench    the default bench line (roofline.traffic from traffic.json) + per-layer table
#   decode   the decode-only line (bench.py --phase decode: decompress of streams encoded before the
#            timed region), same traffic file
#   rocprof  rocprofv3 --kernel-trace --stats of the isolated pass alone (the launches the line's
#            roofline.frac divides by) and of the timed configuration alone
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/record}
KERN=${2:-conv_x4_kernel}
STAGES=${3:-"tests pmc bench decode rocprof"}
ISO="--lanes 1 --batch 8 --split 1"  # (with --no-decode-record below: the main region's launches only)
mkdir -p "$OUT"
export TMPDIR=/tmp
has() { case " $STAGES " in *" $1 "*) return 0;; esac; return 1; }
if has tests; then
  # (no -x: a failing test is recorded with the rest of the suite and the measurements still run;
  # a time limit, abort or crash ends the record)
  MLIC_PARITY_OUT="$OUT/parity_counts.json" timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 \
    --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "tests rc=$rc"; grep -E "^FAILED|^E  " "$OUT/gpu_tests.log" | head -30; fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  tail -1 "$OUT/gpu_tests.log"
fi
if has pmc; then
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 -u bench.py $ISO --steps 1 --warmup 0 --no-cpu-baseline --no-roofline --no-decode-record > "$OUT/pmc_fetch.log" 2>&1 ||
    { echo "pmc fetch failed $?"; tail -20 "$OUT/pmc_fetch.log"; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 -u bench.py $ISO --steps 1 --warmup 0 --no-cpu-baseline --no-roofline --no-decode-record > "$OUT/pmc_write.log" 2>&1 ||
    { echo "pmc write failed $?"; tail -20 "$OUT/pmc_write.log"; exit 1; }
  python3 tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" "$KERN" "$OUT/traffic.json" config=main \
    "launches_of=isolated pass: bench.py --lanes 1 --batch 8 --split 1 --steps 1 --warmup 0 (the launches roofline.frac divides by)" || exit 1
  rm -rf "$OUT/pmc_fetch" "$OUT/pmc_write"
fi
if has bench; then
  TJ="$OUT/traffic.json"; [ -f "$TJ" ] || TJ=profiles/traffic_r06.json
  timeout -k 10 600 python3 -u bench.py --traffic-json "$TJ" --layers-out "$OUT/layers.tsv" \
    > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed $?"; tail -30 "$OUT/bench.err"; exit 1; }
  head -c 400 "$OUT/bench.json"; echo
fi
if has decode; then
  TJ="$OUT/traffic.json"; [ -f "$TJ" ] || TJ=profiles/traffic_r06.json
  timeout -k 10 600 python3 -u bench.py --phase decode --traffic-json "$TJ" > "$OUT/bench_decode.json" \
    2> "$OUT/bench_decode.err" || { echo "bench decode failed $?"; tail -30 "$OUT/bench_decode.err"; exit 1; }
  head -c 300 "$OUT/bench_decode.json"; echo
fi
if has rocprof; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_iso" -o run -- \
    python3 -u bench.py $ISO --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-decode-record > "$OUT/bench_iso_under_rocprof.json" \
    2> "$OUT/rocprof_iso.err" || { echo "rocprof iso failed $?"; tail -20 "$OUT/rocprof_iso.err"; exit 1; }
  rm -f "$OUT"/prof_iso/run_kernel_trace.csv
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_timed" -o run -- \
    python3 -u bench.py --no-cpu-baseline --no-roofline --no-decode-record > "$OUT/bench_timed_under_rocprof.json" \
    2> "$OUT/rocprof_timed.err" || { echo "rocprof timed failed $?"; tail -20 "$OUT/rocprof_timed.err"; exit 1; }
  rm -f "$OUT"/prof_timed/run_kernel_trace.csv
fi
echo "record done"
