cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/diff
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 0 --layers-out gpurun_out/diff/plain.tsv > gpurun_out/diff/plain.json 2>/dev/null || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/diff/prof -o run -- python bench.py --no-cpu-baseline --steps 1 --warmup 0 --layers-out gpurun_out/diff/rocprof.tsv > gpurun_out/diff/rocprof.json 2>/dev/null || exit 1
echo ok
