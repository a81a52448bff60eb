# round 6: compress skips the last slice's non-anchor LRP: coder / round-trip tests
cd "$GRAFT_REPO_ROOT"; OUT=${OUT:-gpurun_out/r6ls}; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "roundtrip or narrow or batched or rate or ep_half or coder or interop or vbr or 1080 or kodak" > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error" $OUT/tests.log | head; exit $rc; }
