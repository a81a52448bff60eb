# round 6: LocalContext attention staging (one cell x 48 channels per thread) vs the element-per-thread form
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6la; mkdir -p $OUT
OLD=$PWD/mlic_amd/libmlic_hip_la0.so
for rep in 1 2 3; do
  MLIC_HIP_LIB=$OLD timeout -k 10 60 python3 tools/gpu/attn_packed_bench.py 8 | sed 's/^/la0 /' || exit 1
  timeout -k 10 60 python3 tools/gpu/attn_packed_bench.py 8 | sed 's/^/new /' || exit 1
done
MLIC_HIP_LIB=$OLD timeout -k 10 60 python3 tools/gpu/la_hash.py | sed 's/^/la0 /' || exit 1
timeout -k 10 60 python3 tools/gpu/la_hash.py | sed 's/^/new /' || exit 1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_conv.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "local or forward_matches or module_vectors" > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT ARGS="--no-decode-record" REPS=2 STEPS=4 bash tools/gpu/ab_env.sh "MLIC_HIP_LIB=$OLD"
