# alternating A/B on the main config: default vs no hoisted EP hyper GEMM vs 8 request streams x 1 lane
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/ab3; mkdir -p $OUT
run() { tag=$1; shift; env "$@" timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline $ARGS > $OUT/b.json 2> $OUT/b.err || { echo "$tag fail"; tail -5 $OUT/b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b.json').readline()); print('$tag', d['value'], d['ms_per_step'])"; }
for rep in 1 2; do
  ARGS="" run default MLIC_HOIST=1 || exit 1
  ARGS="" run hoist0 MLIC_HOIST=0 || exit 1
  ARGS="--split 8 --lanes 1" run s8l1 MLIC_HOIST=1 || exit 1
  ARGS="--split 4 --lanes 3" run s4l3 MLIC_HOIST=1 || exit 1
done
