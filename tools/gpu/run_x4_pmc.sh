cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_LDS --kernel-include-regex conv_x4_kernel -f csv -d gpurun_out/x4pmc1 -o run -- python tools/conv_one.py 7 8 192 768 272 480 3 1 1 3 > gpurun_out/x4pmc1.log 2>&1 || { echo "pmc1 failed $?"; tail -5 gpurun_out/x4pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex conv_x4_kernel -f csv -d gpurun_out/x4pmc2 -o run -- python tools/conv_one.py 7 8 192 768 272 480 3 1 1 3 > gpurun_out/x4pmc2.log 2>&1 || { echo "pmc2 failed $?"; tail -5 gpurun_out/x4pmc2.log; exit 1; }
timeout -k 10 400 python -u bench.py --no-cpu-baseline --profile-lanes 1 --layers-out gpurun_out/layers_x4.tsv > gpurun_out/bench_x4.json 2> gpurun_out/bench_x4.err || { echo "bench failed $?"; tail -30 gpurun_out/bench_x4.err; exit 1; }
cat gpurun_out/bench_x4.json
