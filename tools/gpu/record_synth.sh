# The reduced-precision synthesis line: default workload with g_s subpel convs on fp16
# operands; usage on the box:  bash tools/gpu/record_synth.sh <outdir>
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/r02}
mkdir -p "$OUT"
timeout -k 10 400 python3 -u bench.py --synth-fp16 --no-cpu-baseline --layers-out "$OUT/layers_synth_fp16.tsv" \
  > "$OUT/bench_synth_fp16.json" 2> "$OUT/bench_synth_fp16.err" ||
  { echo "bench synth-fp16 failed $?"; tail -20 "$OUT/bench_synth_fp16.err"; exit 1; }
head -c 400 "$OUT/bench_synth_fp16.json"
