cd "$GRAFT_REPO_ROOT"
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -m pytest tests/test_gpu_conv.py -q -m gpu > gpurun_out/conv_tests_19.log 2>&1
rc=$?; echo "conv tests rc=$rc" >> gpurun_out/conv_tests_19.log; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python tools/conv_bench.py 2 6 > gpurun_out/conv_bench_19.log 2>&1 || exit $?
echo done
