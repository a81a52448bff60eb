cd "$GRAFT_REPO_ROOT"
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -m pytest tests/test_gpu_conv.py -q -m gpu > gpurun_out/conv_tests_15.log 2>&1
rc=$?; echo "conv tests rc=$rc" >> gpurun_out/conv_tests_15.log; if fatal $rc; then exit $rc; fi
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu > gpurun_out/gpu_tests_15.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/gpu_tests_15.log; if fatal $rc; then exit $rc; fi
b() { timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 "$@"; }
b --lanes 4 --layers-out gpurun_out/layers_15.tsv > gpurun_out/b15_b8.json 2>>gpurun_out/b15.err || exit $?
b --lanes 4 --batch 16 --layers-out gpurun_out/layers_15_b16.tsv > gpurun_out/b15_b16.json 2>>gpurun_out/b15.err || exit $?
b --lanes 4 --batch 24 > gpurun_out/b15_b24.json 2>>gpurun_out/b15.err || exit $?
b --lanes 6 --batch 24 > gpurun_out/b15_b24_l6.json 2>>gpurun_out/b15.err || exit $?
b --lanes 4 --batch 32 > gpurun_out/b15_b32.json 2>>gpurun_out/b15.err || exit $?
echo done
