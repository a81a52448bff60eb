# round 6: EntropyParameters chains on their phase's checkerboard half (default) vs the whole grid (MLIC_EP_HALF=0)
cd "$GRAFT_REPO_ROOT"; OUT=${OUT:-gpurun_out/r6eh}; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_conv.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "ep_half or chain or forward_matches or roundtrip or module_vectors or narrow or vbr or batched or local" > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error" $OUT/tests.log | head; exit $rc; }
OUT=$OUT ARGS="--no-decode-record" REPS=2 STEPS=4 bash tools/gpu/ab_env.sh "MLIC_EP_HALF=0" || exit 1
OUT=$OUT CONFIG=vbr-mixed REPS=1 STEPS=3 bash tools/gpu/ab_env.sh "MLIC_EP_HALF=0"
