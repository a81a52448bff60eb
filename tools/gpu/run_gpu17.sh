cd "$GRAFT_REPO_ROOT"
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -m pytest tests/test_gpu_conv.py -q -m gpu > gpurun_out/conv_tests_17.log 2>&1
rc=$?; echo "conv tests rc=$rc" >> gpurun_out/conv_tests_17.log; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python tools/conv_bench.py 6 > gpurun_out/conv_bench_17.log 2>&1 || exit $?
MLIC_HALO_WIDE=0 timeout -k 10 300 python tools/conv_bench.py 6 > gpurun_out/conv_bench_17_narrow.log 2>&1 || exit $?
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu > gpurun_out/gpu_tests_17.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/gpu_tests_17.log; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --batch 16 --layers-out gpurun_out/layers_17.tsv > gpurun_out/b17_b16.json 2>gpurun_out/b17.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --batch 24 > gpurun_out/b17_b24.json 2>>gpurun_out/b17.err || exit $?
echo done
