# GPU tests (with parity counts) + the default bench line with its per-layer table.
#   bash tools/gpu/r3_check.sh <outdir> [pytest -k expr]
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/check}
K=${2:-}
mkdir -p "$OUT"
export TMPDIR=/tmp
export MLIC_PARITY_OUT="$OUT/parity_counts.json"
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${KA[@]}" > "$OUT/gpu_tests.log" 2>&1 || { echo "tests failed $?"; tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -3 "$OUT/gpu_tests.log"
timeout -k 10 600 python -u bench.py --no-cpu-baseline --layers-out "$OUT/layers.tsv" > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed $?"; tail -30 "$OUT/bench.err"; exit 1; }
head -c 700 "$OUT/bench.json"
