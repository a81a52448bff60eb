cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/gpu_tests_4.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/gpu_tests_4.log
if fatal $rc; then exit $rc; fi
for L in 1 2 4; do
  MLIC_LANES=$L timeout -k 10 600 python bench.py --batch 4 --no-cpu-baseline > gpurun_out/bench_4_l$L.json 2> gpurun_out/bench_4_l$L.err || exit $?
done
MLIC_LANES=4 timeout -k 10 600 python bench.py --batch 8 --no-cpu-baseline > gpurun_out/bench_4_b8.json 2> gpurun_out/bench_4_b8.err || exit $?
echo all-done
