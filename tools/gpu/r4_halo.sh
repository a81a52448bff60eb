# x4 halo-staged B: kernel tests, then the conv micro-benchmark with the halo off / on
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/halo}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread -k "x4" \
  > "$OUT/conv_tests.log" 2>&1 || { echo "conv tests failed $?"; tail -30 "$OUT/conv_tests.log"; exit 1; }
tail -1 "$OUT/conv_tests.log"
for h in 0 1; do
  MLIC_X4_HALO=$h timeout -k 10 200 python3 -u tools/gpu/bench_conv.py > "$OUT/bench_halo$h.log" 2>&1 ||
    { echo "bench halo=$h failed $?"; tail -20 "$OUT/bench_halo$h.log"; exit 1; }
  echo "halo=$h"; cat "$OUT/bench_halo$h.log"
done
