cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 120 --timeout-method thread -k "narrow or auto" > gpurun_out/nr_tests.log 2>&1 || { echo "tests failed $?"; grep -E "^E|FAILED" gpurun_out/nr_tests.log | head; exit 1; }
tail -1 gpurun_out/nr_tests.log
timeout -k 10 120 python tools/conv_one.py 4 8 192 12 544 960 3 1 1 10 || exit 1
