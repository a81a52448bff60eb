cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 120 --timeout-method thread -k "x4 or auto" > gpurun_out/x4_tests.log 2>&1 || { echo "x4 tests failed $?"; tail -40 gpurun_out/x4_tests.log; exit 1; }
tail -2 gpurun_out/x4_tests.log
for a in 0 4; do
  echo "abl=$a"; MLIC_X4_ABL=$a timeout -k 10 120 python tools/conv_one.py 7 8 192 768 272 480 3 1 1 10 || exit 1
done
timeout -k 10 120 python tools/conv_one.py 7 8 192 768 136 240 3 1 1 10 || exit 1
timeout -k 10 120 python tools/conv_one.py 7 8 480 1920 34 60 3 1 1 10 || exit 1
