cd "$GRAFT_REPO_ROOT"
for b in 16 32 48; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch $b --steps 2 > gpurun_out/bench_b$b.json 2> gpurun_out/bench_b$b.err || { echo "bench $b failed $?"; tail -5 gpurun_out/bench_b$b.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_b$b.json')); print($b, d['value'], d['ms_per_step'], d['gpu_kernel_ms_per_step_isolated'])"
done
for l in 2 3 6; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch 24 --lanes $l --steps 2 > gpurun_out/bench_l$l.json 2> gpurun_out/bench_l$l.err || { echo "bench l$l failed $?"; tail -5 gpurun_out/bench_l$l.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_l$l.json')); print('lanes', $l, d['value'], d['ms_per_step'])"
done
