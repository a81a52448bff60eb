# GPU tests (with exact parity counts) + the default bench line; usage on the box:
#   bash tools/gpu/check.sh <outdir>
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/check}
mkdir -p "$OUT"
export TMPDIR=/tmp
export MLIC_PARITY_OUT="$OUT/parity_counts.json"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { echo "tests failed $?"; tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -3 "$OUT/gpu_tests.log"
timeout -k 10 600 python -u bench.py --layers-out "$OUT/layers.tsv" > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed $?"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
