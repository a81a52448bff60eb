cd "$GRAFT_REPO_ROOT"
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -m pytest tests/test_gpu_conv.py -q -m gpu -x > gpurun_out/conv_tests_14.log 2>&1
rc=$?; echo "conv tests rc=$rc" >> gpurun_out/conv_tests_14.log; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python tools/conv_bench.py 2 6 3 > gpurun_out/conv_bench_14.log 2>&1 || exit $?
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu > gpurun_out/gpu_tests_14.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/gpu_tests_14.log; if fatal $rc; then exit $rc; fi
b() { timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 "$@"; }
b --lanes 4 --layers-out gpurun_out/layers_14.tsv > gpurun_out/b14_l4.json 2>>gpurun_out/b14.err || exit $?
b --lanes 8 > gpurun_out/b14_l8.json 2>>gpurun_out/b14.err || exit $?
MLIC_LANE_PRIORITY=0 b --lanes 4 > gpurun_out/b14_l4_noprio.json 2>>gpurun_out/b14.err || exit $?
b --lanes 4 --batch 16 > gpurun_out/b14_l4_b16.json 2>>gpurun_out/b14.err || exit $?
b --lanes 8 --batch 16 > gpurun_out/b14_l8_b16.json 2>>gpurun_out/b14.err || exit $?
echo done
