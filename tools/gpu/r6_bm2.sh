# round 6: x4 tile height, h_s 480 -> 640 1x1 at 34 x 60 (isolated), then parity tests and the main line with the new 1280 rule
cd "$GRAFT_REPO_ROOT"; OUT=${OUT:-gpurun_out/r6bm2}; mkdir -p $OUT
SH="8 480 640 34 60 1 1 0 8 320 1280 17 30 3 1 129"
for rep in 1 2; do
  for arm in "" "640:256" "640:192" "1280:256"; do
    echo "== [$arm]"
    MLIC_X4_BM_FOR="$arm" timeout -k 10 120 python3 tools/gpu/bench_conv.py $SH || exit 1
  done
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_conv.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "x4 or forward_matches or roundtrip or module_vectors or rate or batched" > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error" $OUT/tests.log | head; exit $rc; }
OUT=$OUT ARGS="--no-decode-record" REPS=2 STEPS=4 bash tools/gpu/ab_env.sh "MLIC_X4_BM_FOR=1280:256"
