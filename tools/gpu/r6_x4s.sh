# round 6: x4 staggered staging A/B (product library vs -DMLIC_X4_STAGGER=0 build), then x4 / model tests
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6s; mkdir -p $OUT
SH="8 192 768 272 480 3 1 129 8 192 768 136 240 3 1 128 8 288 96 68 120 5 1 0 8 480 1920 34 60 3 1 129 8 32 64 68 120 5 1 0"
for rep in 1 2 3; do
for v in s0 "" h3; do
  unset MLIC_X4_HALO
  if [ "$v" = s0 ]; then export MLIC_HIP_LIB=$PWD/mlic_amd/libmlic_hip_x4$v.so; else unset MLIC_HIP_LIB; fi
  if [ "$v" = h3 ]; then export MLIC_X4_HALO=2; fi
  echo "== lib=${v:-stagger} rep $rep"
  timeout -k 10 120 python3 tools/gpu/bench_conv.py $SH || exit 1
done; done
unset MLIC_X4_HALO
unset MLIC_HIP_LIB
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_conv.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "x4 or forward_matches or roundtrip or module_vectors or 1080 or reprojection or halo" > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT ARGS="--no-decode-record" REPS=2 STEPS=4 bash tools/gpu/ab_env.sh "MLIC_HIP_LIB=$PWD/mlic_amd/libmlic_hip_x4s0.so" "MLIC_X4_HALO=2"
