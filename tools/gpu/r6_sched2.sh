# round 6: join vs streams schedule of the request streams, main line, 4 alternating pairs
cd "$GRAFT_REPO_ROOT"; OUT=${OUT:-gpurun_out/r6s2}; mkdir -p $OUT
OUT=$OUT ARGS="--no-decode-record" REPS=4 STEPS=4 bash tools/gpu/ab_env.sh "MLIC_SCHEDULE=streams"
