# round 6: halo-form x4 with two taps per K-step (default) vs one (-DMLIC_X4_TPS=1): 5x5 reprojections, tests, main line
cd "$GRAFT_REPO_ROOT"; OUT=${OUT:-gpurun_out/r6tps}; mkdir -p $OUT
SH="8 288 96 68 120 5 1 0 8 160 96 68 120 5 1 0 8 32 64 68 120 5 1 0"
for rep in 1 2; do
for v in tps1 new; do
  if [ $v = new ]; then unset MLIC_HIP_LIB; else export MLIC_HIP_LIB=$PWD/mlic_amd/libmlic_hip_$v.so; fi
  echo "== $v rep $rep"
  timeout -k 10 120 python3 tools/gpu/bench_conv.py $SH || exit 1
done; done
unset MLIC_HIP_LIB
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_conv.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "x4 or halo or forward_matches or roundtrip or module_vectors or 1080 or range or split" > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error" $OUT/tests.log | head; exit $rc; }
OUT=$OUT ARGS="--no-decode-record" REPS=2 STEPS=4 bash tools/gpu/ab_env.sh "MLIC_HIP_LIB=$PWD/mlic_amd/libmlic_hip_tps1.so"
