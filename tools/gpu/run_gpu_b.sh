cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'conv_x3v2_kernelILi256ELi256E' -f csv -d gpurun_out/pmc_fetch -o run -- python -X faulthandler bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_fetch.log 2>&1 || { echo "fetch failed $?"; grep -v '^    @' gpurun_out/pmc_fetch.log | tail -30; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'conv_x3v2_kernelILi256ELi256E' -f csv -d gpurun_out/pmc_write -o run -- python -X faulthandler bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_write.log 2>&1 || { echo "write failed $?"; grep -v '^    @' gpurun_out/pmc_write.log | tail -30; exit 1; }
python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write conv_x3v2_kernelILi256ELi256E gpurun_out/traffic.json model=MLICPP_L H=1088 W=1920 batch=24 'family=conv_x3v2_kernel<256,256>' || exit 1
echo done
