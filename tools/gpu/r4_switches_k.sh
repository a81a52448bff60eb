# Kodak-size config: split-K off vs default, alternating
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/swk; mkdir -p $OUT
run() { tag=$1; env $tag timeout -k 10 300 python3 -u bench.py --config ${CFG:-kodak} --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > $OUT/b.json 2> $OUT/b.err || { echo "$tag fail"; tail -5 $OUT/b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b.json').readline()); print('${CFG:-kodak} $tag', d['value'], d['ms_per_step'])"; }
for rep in 1 2; do run MLIC_DEFAULT=1 && run MLIC_X4_SPLITK=0 || exit 1; done
