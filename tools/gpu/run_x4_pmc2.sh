cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
S="python tools/conv_one.py 7 8 192 768 272 480 3 1 1 3"
p() { timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex conv_x4_kernel -f csv -d gpurun_out/x4p_$1 -o run -- $S > gpurun_out/x4p_$1.log 2>&1 || { echo "pmc $1 failed $?"; tail -5 gpurun_out/x4p_$1.log; exit 1; }; }
p SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES
p TCC_HIT_sum TCC_MISS_sum
p TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
p TA_BUSY_avr TA_TA_BUSY_sum
echo done
