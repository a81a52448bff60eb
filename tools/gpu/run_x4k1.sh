cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 120 --timeout-method thread -k "x4 or auto" > gpurun_out/x4_tests.log 2>&1 || { echo "x4 tests failed $?"; tail -40 gpurun_out/x4_tests.log; exit 1; }
tail -2 gpurun_out/x4_tests.log
for shp in "960 320" "832 320" "704 320" "640 320" "320 256" "256 128" "608 224" "352 224" "224 128" "128 64"; do
  for impl in 3 7; do
    timeout -k 10 120 python tools/conv_one.py $impl 6 $shp 68 120 1 1 0 20 || exit 1
  done
done
