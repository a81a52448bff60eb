cd "$GRAFT_REPO_ROOT"
MLIC_LANE_PRIORITY=0 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "conv_x3v2_kernel" -f csv -d gpurun_out/pmc23_a -o run -- python -X faulthandler bench.py --steps 1 --warmup 0 --no-cpu-baseline --lanes 1 --batch 2 > gpurun_out/pmc23_a.log 2>&1 || { echo "a failed $?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "conv_x3v2_kernel" -f csv -d gpurun_out/pmc23_b -o run -- python -X faulthandler bench.py --steps 1 --warmup 0 --no-cpu-baseline --lanes 2 --batch 2 > gpurun_out/pmc23_b.log 2>&1 || { echo "b failed $?"; exit 1; }
echo done
