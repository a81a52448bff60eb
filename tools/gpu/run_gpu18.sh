cd "$GRAFT_REPO_ROOT"
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
MLIC_V2_WIDE=1 timeout -k 10 300 python -m pytest tests/test_gpu_conv.py -q -m gpu -k "generic or auto" > gpurun_out/conv_tests_18.log 2>&1
rc=$?; echo "conv tests rc=$rc" >> gpurun_out/conv_tests_18.log; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python tools/conv_bench.py 2 > gpurun_out/conv_bench_18.log 2>&1 || exit $?
MLIC_V2_WIDE=1 timeout -k 10 300 python tools/conv_bench.py 2 > gpurun_out/conv_bench_18_wide.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --batch 16 > gpurun_out/b18_b16.json 2>gpurun_out/b18.err || exit $?
MLIC_V2_WIDE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --batch 16 > gpurun_out/b18_b16_wide.json 2>>gpurun_out/b18.err || exit $?
echo done
