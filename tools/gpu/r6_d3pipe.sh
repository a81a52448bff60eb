# round 6: dwpw3 consumer block order A/B: new (both blocks' MFMAs, then both epilogues; RES forms restructured)
# vs -DMLIC_D3_PIPE=0 vs the previous head's dwpw3; alternating, one box; then dwpw tests and the model line
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6d; mkdir -p $OUT
for rep in 1 2 3; do
for v in old p0 new; do
  if [ $v = new ]; then unset MLIC_HIP_LIB; else export MLIC_HIP_LIB=$PWD/mlic_amd/libmlic_hip_d3$v.so; fi
  for epi in 1 0 65; do echo -n "$v rep $rep "; timeout -k 10 120 python3 tools/gpu/bench_dwpw.py 8 192 544 960 $epi 2>&1 | grep fused || exit 1; done
done; done
unset MLIC_HIP_LIB
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 300 --timeout-method thread -k "dwpw or pw3" > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT ARGS="--no-decode-record" REPS=2 STEPS=4 bash tools/gpu/ab_env.sh "MLIC_HIP_LIB=$PWD/mlic_amd/libmlic_hip_d3old.so"
