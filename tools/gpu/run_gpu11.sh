# lanes sweep, then rocprofv3 kernel stats of the default bench command and PMC traffic passes
cd "$GRAFT_REPO_ROOT"
for L in 2 8 4; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --lanes $L > gpurun_out/bench_11_l$L.json 2>>gpurun_out/bench_11.err || exit $?
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof11 -o run -- python bench.py --no-cpu-baseline > gpurun_out/prof11.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "conv_x3v2|pw_resident" -f csv -d gpurun_out/pmc_fetch11 -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_fetch11.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "conv_x3v2|pw_resident" -f csv -d gpurun_out/pmc_write11 -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_write11.log 2>&1 || exit $?
echo done
