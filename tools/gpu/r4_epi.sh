# epilogue / raster changes: the kernel tests that pin them, the conv micro-benchmark, the bench line
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/epi}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread \
  -k "dwpw or pw_resident or x4 or auto" > "$OUT/conv_tests.log" 2>&1 || { echo "conv tests failed $?"; tail -30 "$OUT/conv_tests.log"; exit 1; }
tail -1 "$OUT/conv_tests.log"
timeout -k 10 200 python3 -u tools/gpu/bench_conv.py > "$OUT/bench_conv.log" 2>&1 || { echo "bench_conv failed"; exit 1; }
grep impl "$OUT/bench_conv.log"
timeout -k 10 200 python3 -u tools/gpu/bench_dwpw.py > "$OUT/bench_dwpw.log" 2>&1 || { echo "bench_dwpw failed"; tail -5 "$OUT/bench_dwpw.log"; }
tail -8 "$OUT/bench_dwpw.log"
bash tools/gpu/r4_quick.sh "$OUT/q" "roundtrip or module_vectors"
