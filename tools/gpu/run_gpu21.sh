# round-1 profiling artefacts: PMC traffic of the dominant kernel, then rocprofv3 kernel stats of
# the default bench command (whose JSON line then carries the PMC traffic)
cd "$GRAFT_REPO_ROOT"
K="conv_x3v2_kernel<256,256"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "conv_x3v2_kernel<256" -f csv -d gpurun_out/pmc_fetch21 -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_fetch21.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "conv_x3v2_kernel<256" -f csv -d gpurun_out/pmc_write21 -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_write21.log 2>&1 || exit $?
python tools/pmc_traffic.py gpurun_out/pmc_fetch21 gpurun_out/pmc_write21 "$K" profiles/traffic_r01.json model=MLICPP_L H=1088 W=1920 batch=24 > gpurun_out/traffic21.log 2>&1 || exit $?
timeout -k 10 900 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof21 -o run -- python bench.py > gpurun_out/prof21.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --no-cpu-baseline --profile-lanes 1 --layers-out gpurun_out/layers_21.tsv > gpurun_out/b21_isolated.json 2> gpurun_out/b21.err || exit $?
echo done
