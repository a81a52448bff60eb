cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed $?"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
b() { timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --layers-out gpurun_out/ab_$1.tsv > gpurun_out/ab_$1.json 2>gpurun_out/ab_$1.err || exit 1; python -c "import json; d=json.load(open('gpurun_out/ab_$1.json')); print('$1', d['value'], d['ms_per_step'], d['gpu_kernel_ms_isolated_share'], d['roofline']['frac'])"; }
b k3
MLIC_X4_K=13 b k13
MLIC_X4_K=135 b k135
b k3b
