cd "$GRAFT_REPO_ROOT"
p() { timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "conv_x3v2_kernel" -f csv -d gpurun_out/pmc22_$1 -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline "${@:2}" > gpurun_out/pmc22_$1.log 2>&1; }
p a --lanes 1 --batch 2 || { echo "a failed $?"; exit 1; }
MLIC_LANE_PRIORITY=0 p b --lanes 2 --batch 2 || { echo "b failed $?"; exit 1; }
p c --lanes 2 --batch 2 || { echo "c failed $?"; exit 1; }
echo done
