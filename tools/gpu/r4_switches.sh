# alternating A/B of the environment switches at the current head (main config, timed steps only)
# usage: bash tools/gpu/r4_switches.sh "VAR=VAL VAR2=VAL2 ..."  (each a separate arm, plus the default)
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/sw; mkdir -p $OUT
run() { tag=$1; env $tag timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > $OUT/b.json 2> $OUT/b.err || { echo "$tag fail"; tail -5 $OUT/b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b.json').readline()); print('$tag', d['value'], d['ms_per_step'])"; }
for rep in 1 2; do
  run MLIC_DEFAULT=1 || exit 1
  for a in $1; do run $a || exit 1; done
done
