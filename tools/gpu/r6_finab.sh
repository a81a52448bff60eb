# round 6: final head vs the record head (before the 1280-row rule and the compress LRP skip), main line, alternating
cd "$GRAFT_REPO_ROOT"; OUT=${OUT:-gpurun_out/r6fab}; mkdir -p $OUT
OUT=$OUT ARGS="--no-decode-record" REPS=3 STEPS=4 bash tools/gpu/ab_env.sh "MLIC_HIP_LIB=$PWD/mlic_amd/libmlic_hip_prev.so"
