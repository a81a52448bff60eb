# Kernel trace of the timed configuration (no profiled passes) for the GPU-occupancy analysis of
# tools/trace_busy.py; usage on the box: bash tools/gpu/busy_trace.sh <outdir> [bench args]
cd "$GRAFT_REPO_ROOT"; OUT=${1:-gpurun_out/busy}; shift; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr" -o run -- \
  python3 -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-roofline "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" ||
  { echo "trace failed $?"; tail "$OUT/bench.err"; exit 1; }
f=$(ls "$OUT"/tr/*kernel_trace.csv "$OUT"/tr/*/*kernel_trace.csv 2>/dev/null | head -1)
gzip -c "$f" > "$OUT/kernel_trace.csv.gz" && rm -rf "$OUT/tr"
python3 tools/trace_busy.py <(zcat "$OUT/kernel_trace.csv.gz") 0.2
