cd "$GRAFT_REPO_ROOT"
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python tools/conv_bench.py 0 1 2 > gpurun_out/conv_bench_9.log 2>&1 || exit $?
MLIC_PRECISION=2 timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu > gpurun_out/gpu_tests_9.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/gpu_tests_9.log; if fatal $rc; then exit $rc; fi
timeout -k 10 600 python bench.py --precision 2 --no-cpu-baseline --steps 2 --layers-out gpurun_out/layers_9.tsv > gpurun_out/bench_9.json 2> gpurun_out/bench_9.err || exit $?
echo done
