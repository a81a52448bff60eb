set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu > gpurun_out/gpu_tests_2.log 2>&1; echo "tests rc=$?" >> gpurun_out/gpu_tests_2.log
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --batch 2 --no-cpu-baseline > gpurun_out/bench_2.log 2>&1 && echo bench ok
