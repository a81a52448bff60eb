# round record: GPU tests, default bench (with CPU baseline), rocprofv3 kernel stats of the same
# command, PMC FETCH/WRITE passes for the dominant kernel family (conv_x4_kernel)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final/gpu_tests.log 2>&1 || { echo "tests failed $?"; tail -30 gpurun_out/final/gpu_tests.log; exit 1; }
tail -1 gpurun_out/final/gpu_tests.log
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex conv_x4_kernel -f csv -d gpurun_out/final/pmc_fetch -o run -- python bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/final/pmc_fetch.log 2>&1 || { echo "pmc fetch failed $?"; tail -5 gpurun_out/final/pmc_fetch.log; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex conv_x4_kernel -f csv -d gpurun_out/final/pmc_write -o run -- python bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/final/pmc_write.log 2>&1 || { echo "pmc write failed $?"; tail -5 gpurun_out/final/pmc_write.log; exit 1; }
python tools/pmc_traffic.py gpurun_out/final/pmc_fetch gpurun_out/final/pmc_write conv_x4_kernel gpurun_out/final/traffic.json model=MLICPP_L H=1088 W=1920 batch=32 family=conv_x4_kernel || exit 1
cp gpurun_out/final/traffic.json profiles/traffic_r01.json
timeout -k 10 500 python -u bench.py --layers-out gpurun_out/final/layers.tsv > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { echo "bench failed $?"; tail -20 gpurun_out/final/bench.err; exit 1; }
timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/final/prof -o run -- python bench.py --no-cpu-baseline > gpurun_out/final/bench_rocprof.json 2> gpurun_out/final/bench_rocprof.err || { echo "rocprof failed $?"; tail -20 gpurun_out/final/bench_rocprof.err; exit 1; }
cat gpurun_out/final/bench.json
