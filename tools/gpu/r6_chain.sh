# round 6: chain wave-layout A/B (tests, then alternating timed bench arms, then isolated family times)
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6c; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "chain or module_vectors or forward_matches_reference_fixture or lanes_do_not" > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT ARGS="--no-decode-record" REPS=2 STEPS=4 bash tools/gpu/ab_env.sh "MLIC_CHAIN_NJ=2" || exit 1
for nj in 2 1; do
  MLIC_CHAIN_NJ=$nj timeout -k 10 300 python3 -u bench.py --lanes 1 --batch 8 --split 1 --steps 1 --warmup 1 \
    --no-cpu-baseline --no-decode-record > $OUT/iso_$nj.json 2> $OUT/iso_$nj.err || { echo iso failed; tail -5 $OUT/iso_$nj.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/iso_$nj.json').readline()); f=d['kernel_families_ms_isolated_share']; print('nj=$nj chain', f.get('chain_kernel'), 'total', d['gpu_kernel_ms_isolated_share'])"
done
