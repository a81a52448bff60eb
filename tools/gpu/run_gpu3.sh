# GPU run: parity tests, default bench, rocprofv3 kernel stats, PMC traffic passes.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu > gpurun_out/gpu_tests_3.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/gpu_tests_3.log
if fatal $rc; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench_3.json 2> gpurun_out/bench_3.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof3 -o run -- python bench.py --steps 1 --warmup 1 --batch 2 --no-cpu-baseline > gpurun_out/prof3.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex conv_mfma -f csv -d gpurun_out/pmc_fetch3 -o run -- python bench.py --steps 1 --warmup 0 --batch 1 --no-cpu-baseline > gpurun_out/pmc_fetch3.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex conv_mfma -f csv -d gpurun_out/pmc_write3 -o run -- python bench.py --steps 1 --warmup 0 --batch 1 --no-cpu-baseline > gpurun_out/pmc_write3.log 2>&1 || exit $?
echo all-done
