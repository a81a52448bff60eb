cd "$GRAFT_REPO_ROOT"
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -m pytest tests/test_gpu_conv.py -q -m gpu > gpurun_out/conv_tests_20.log 2>&1
rc=$?; echo "conv tests rc=$rc" >> gpurun_out/conv_tests_20.log; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python tools/conv_bench.py 3 > gpurun_out/conv_bench_20.log 2>&1 || exit $?
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu > gpurun_out/gpu_tests_20.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/gpu_tests_20.log; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --batch 16 --layers-out gpurun_out/layers_20.tsv > gpurun_out/b20_b16.json 2>gpurun_out/b20.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --batch 24 > gpurun_out/b20_b24.json 2>>gpurun_out/b20.err || exit $?
echo done
