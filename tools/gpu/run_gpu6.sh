cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
MLIC_PRECISION=1 timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu > gpurun_out/gpu_tests_6_x3.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/gpu_tests_6_x3.log; if fatal $rc; then exit $rc; fi
MLIC_PRECISION=0 timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu > gpurun_out/gpu_tests_6_f32.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/gpu_tests_6_f32.log; if fatal $rc; then exit $rc; fi
timeout -k 10 600 python bench.py --precision 1 --no-cpu-baseline > gpurun_out/bench_6_x3.json 2> gpurun_out/bench_6_x3.err || exit $?
timeout -k 10 600 python bench.py --precision 0 --no-cpu-baseline > gpurun_out/bench_6_f32.json 2> gpurun_out/bench_6_f32.err || exit $?
echo all-done
