# round 6: the 5x5 halo form (134 KB LDS, default) vs per-tap B staging (88 KB) in the timed configuration
cd "$GRAFT_REPO_ROOT"; OUT=${OUT:-gpurun_out/r6h0}; mkdir -p $OUT
OUT=$OUT ARGS="--no-decode-record" REPS=3 STEPS=4 bash tools/gpu/ab_env.sh "MLIC_X4_HALO=0"
