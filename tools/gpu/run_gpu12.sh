cd "$GRAFT_REPO_ROOT"
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -m pytest tests/test_gpu_conv.py -q -m gpu -x > gpurun_out/conv_tests_12.log 2>&1
rc=$?; echo "conv tests rc=$rc" >> gpurun_out/conv_tests_12.log; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python tools/conv_bench.py 2 6 3 7 > gpurun_out/conv_bench_12.log 2>&1 || exit $?
MLIC_PRECISION=3 timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu > gpurun_out/gpu_tests_12.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/gpu_tests_12.log; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --layers-out gpurun_out/layers_12.tsv > gpurun_out/bench_12.json 2> gpurun_out/bench_12.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --precision 3 --layers-out gpurun_out/layers_12p3.tsv > gpurun_out/bench_12p3.json 2>> gpurun_out/bench_12.err || exit $?
for L in 2 8; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --lanes $L > gpurun_out/bench_12_l$L.json 2>>gpurun_out/bench_12.err || exit $?
done
echo done
