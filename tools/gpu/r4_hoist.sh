# GPU suite with the auto hoist policy, then alternating bench A/B (auto vs forced hoist)
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/hoist; mkdir -p $OUT
MLIC_PARITY_OUT=$OUT/parity_counts.json timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "^FAILED|^E  " $OUT/gpu_tests.log | head -20; exit $rc; }
run() { tag=$1; shift; env "$@" timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > $OUT/b.json 2> $OUT/b.err || { echo "$tag fail"; tail -5 $OUT/b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b.json').readline()); print('$tag', d['value'], d['ms_per_step'])"; }
for rep in 1 2; do run auto MLIC_X=0 && run hoist1 MLIC_HOIST=1 || exit 1; done
for rep in 1 2; do
  env timeout -k 10 300 python3 -u bench.py --config sd1080 --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > $OUT/s.json 2>$OUT/s.err || { echo sd fail; tail -3 $OUT/s.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/s.json').readline()); print('sd1080 auto', d['value'])"
done
