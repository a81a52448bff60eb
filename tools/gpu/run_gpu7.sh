cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python bench.py --precision 1 --no-cpu-baseline --steps 1 --layers-out gpurun_out/layers_x3.tsv > gpurun_out/bench_7_x3.json 2> gpurun_out/bench_7.err || exit $?
timeout -k 10 600 python bench.py --precision 0 --no-cpu-baseline --steps 1 --layers-out gpurun_out/layers_f32.tsv > gpurun_out/bench_7_f32.json 2>> gpurun_out/bench_7.err || exit $?
echo done
