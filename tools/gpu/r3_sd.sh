cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/sd}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 120 --timeout-method thread -k "x4" > "$OUT/conv_tests.log" 2>&1 || { echo "conv tests failed"; tail -30 "$OUT/conv_tests.log"; exit 1; }
tail -1 "$OUT/conv_tests.log"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "SMALL_DEC or chain or range" > "$OUT/parity_tests.log" 2>&1 || { echo "parity tests failed"; tail -30 "$OUT/parity_tests.log"; exit 1; }
tail -1 "$OUT/parity_tests.log"
for c in sd1080 kodak-sweep; do
  timeout -k 10 400 python3 -u bench.py --config $c --no-cpu-baseline --records-out "$OUT/records_$c.json" > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || { echo "$c failed"; tail -20 "$OUT/bench_$c.err"; exit 1; }
  echo "$c: $(head -c 250 "$OUT/bench_$c.json")"
done
timeout -k 10 400 python3 -u bench.py --config kodak-sweep --emulate-world 8 --emulate-rank 0 --no-cpu-baseline > "$OUT/bench_kodak-sweep_emu8r0.json" 2> "$OUT/emu.err" || { echo "emu failed"; tail -20 "$OUT/emu.err"; exit 1; }
echo "emu: $(head -c 250 "$OUT/bench_kodak-sweep_emu8r0.json")"
