# x4 A/B on the g_s / h_s / context shapes: LDS-staged A (MLIC_X4_AREG=0) vs A in registers, and the
# fp16-operand form (impl 8); then the x4 / model parity tests.  usage: bash tools/gpu/ab_x4.sh <outdir>
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/ab}
mkdir -p "$OUT"
S="8 192 768 272 480 3 1 128  8 192 768 136 240 3 1 128  8 320 768 68 120 3 1 128  8 480 1920 68 120 3 1 129  8 640 6400 68 120 1 1 0  8 288 96 68 120 5 1 0  8 800 64 68 120 1 1 64"
for areg in 0 1; do
  MLIC_X4_AREG=$areg MLIC_BENCH_IMPL=7 timeout -k 10 120 python3 -u tools/gpu/bench_conv.py $S > "$OUT/x4_areg$areg.log" 2>&1 ||
    { echo "bench areg=$areg failed $?"; tail -5 "$OUT/x4_areg$areg.log"; exit 1; }
  echo "areg=$areg"; cat "$OUT/x4_areg$areg.log"
  MLIC_X4_AREG=$areg MLIC_BENCH_IMPL=8 timeout -k 10 120 python3 -u tools/gpu/bench_conv.py 8 192 768 272 480 3 1 128 8 192 768 136 240 3 1 128 \
    > "$OUT/x4h_areg$areg.log" 2>&1 || { echo "bench hi areg=$areg failed $?"; tail -5 "$OUT/x4h_areg$areg.log"; exit 1; }
  cat "$OUT/x4h_areg$areg.log"
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_conv.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  > "$OUT/tests.log" 2>&1 || { echo "tests failed $?"; tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
