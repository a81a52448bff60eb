# round 6: host rANS (dominant-symbol decode fast path, right-sized encoder buffer) vs the previous coder,
# alternating on one box: the VBR 4K + 1080p mix (host-decode-bound) and the main config
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6r; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_lib_cpu.py -q -x -k rans > $OUT/cpu_tests.log 2>&1 || { tail -5 $OUT/cpu_tests.log; exit 1; }
python3 tools/rans_time.py > $OUT/rans_time_new.log 2>&1; MLIC_HIP_LIB=$PWD/mlic_amd/libmlic_hip_rold.so python3 tools/rans_time.py > $OUT/rans_time_old.log 2>&1
cat $OUT/rans_time_old.log $OUT/rans_time_new.log
CONFIG=vbr-mixed OUT=$OUT ARGS="--no-decode-record" REPS=3 STEPS=4 bash tools/gpu/ab_env.sh "MLIC_HIP_LIB=$PWD/mlic_amd/libmlic_hip_rold.so" || exit 1
OUT=$OUT ARGS="--no-decode-record" REPS=2 STEPS=4 bash tools/gpu/ab_env.sh "MLIC_HIP_LIB=$PWD/mlic_amd/libmlic_hip_rold.so"
