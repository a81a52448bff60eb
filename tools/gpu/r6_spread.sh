# round 6: x4 staging spread over the step's pixel groups (product) vs all after group 0 (-DMLIC_X4_SPREAD=0)
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6p; mkdir -p $OUT
SH="8 192 768 272 480 3 1 129 8 192 768 136 240 3 1 128 8 480 1920 34 60 3 1 129 8 288 96 68 120 5 1 0 8 320 1280 17 30 3 1 129"
for rep in 1 2 3; do
for v in sp0 new; do
  if [ $v = new ]; then unset MLIC_HIP_LIB; else export MLIC_HIP_LIB=$PWD/mlic_amd/libmlic_hip_$v.so; fi
  echo "== $v rep $rep"
  timeout -k 10 120 python3 tools/gpu/bench_conv.py $SH || exit 1
done; done
unset MLIC_HIP_LIB
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_conv.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "x4 or forward_matches or roundtrip or module_vectors or 1080 or halo or range" > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT ARGS="--no-decode-record" REPS=2 STEPS=4 bash tools/gpu/ab_env.sh "MLIC_HIP_LIB=$PWD/mlic_amd/libmlic_hip_sp0.so"
