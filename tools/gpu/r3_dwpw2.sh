# fused dwpw A/B: bit-exactness tests (pixel-pair default + lane-per-pixel), micro-benchmark of both
# forms at the full-resolution shapes, then (optional 2nd arg "full") the GPU suite and the default
# bench line with and without the fused path.   bash tools/gpu/r3_dwpw2.sh <outdir> [full]
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/dwpw2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -v --timeout 120 --timeout-method thread -k dwpw > "$OUT/dwpw_test.log" 2>&1 || { echo "dwpw test failed $?"; tail -40 "$OUT/dwpw_test.log"; exit 1; }
tail -2 "$OUT/dwpw_test.log"
MLIC_DWPW_V=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 120 --timeout-method thread -k dwpw > "$OUT/dwpw_test_v1.log" 2>&1 || { echo "dwpw v1 test failed $?"; tail -40 "$OUT/dwpw_test_v1.log"; exit 1; }
tail -1 "$OUT/dwpw_test_v1.log"
for v in 2 1; do
for shp in "8 192 544 960" "8 192 272 480" "8 192 136 240" "8 96 544 960" "8 128 544 960"; do
  MLIC_DWPW_V=$v timeout -k 10 120 python -u tools/gpu/bench_dwpw.py $shp > "$OUT/b.tmp" 2>&1 || { echo "bench_dwpw failed"; cat "$OUT/b.tmp"; exit 1; }
  echo "v$v $(grep fused "$OUT/b.tmp")" >> "$OUT/bench_dwpw.log"
done
done
cat "$OUT/bench_dwpw.log"
if [ "$2" = "full" ]; then
  bash tools/gpu/r3_check.sh "$OUT" || exit 1
  MLIC_DWPW=1 timeout -k 10 600 python -u bench.py --no-cpu-baseline --layers-out "$OUT/layers_dwpw.tsv" > "$OUT/bench_dwpw_on.json" 2> "$OUT/bench_dwpw_on.err" || { echo "bench dwpw failed $?"; tail -30 "$OUT/bench_dwpw_on.err"; exit 1; }
  head -c 400 "$OUT/bench_dwpw_on.json"
fi
