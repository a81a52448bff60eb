# quick GPU gate after a kernel change: conv-kernel tests (+ optional -k expr), the parity tests that
# pin the model (fixtures, rate sets, round trips), then the default bench line with its layer table.
#   bash tools/gpu/r3_quick.sh <outdir> [conv -k expr]
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/quick}
mkdir -p "$OUT"
export TMPDIR=/tmp
export MLIC_PARITY_OUT="$OUT/parity_counts.json"
if [ -n "$2" ]; then KA=(-k "$2"); else KA=(); fi
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 120 --timeout-method thread "${KA[@]}" > "$OUT/conv_tests.log" 2>&1 || { echo "conv tests failed $?"; tail -40 "$OUT/conv_tests.log"; exit 1; }
tail -1 "$OUT/conv_tests.log"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "fixture or rate_sets or roundtrip or streams or kodak" > "$OUT/parity_tests.log" 2>&1 || { echo "parity tests failed $?"; tail -40 "$OUT/parity_tests.log"; exit 1; }
tail -1 "$OUT/parity_tests.log"
timeout -k 10 600 python -u bench.py --no-cpu-baseline --layers-out "$OUT/layers.tsv" > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed $?"; tail -30 "$OUT/bench.err"; exit 1; }
head -c 300 "$OUT/bench.json"; echo
