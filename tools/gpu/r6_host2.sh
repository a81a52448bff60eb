# round 6: request streams x lanes under the streams schedule, main line, alternating arms on one box
cd "$GRAFT_REPO_ROOT"; OUT=${OUT:-gpurun_out/r6h2}; mkdir -p $OUT
run() {
  timeout -k 10 300 python3 -u bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-roofline --no-decode-record $1 > $OUT/b.json 2> $OUT/b.err || { echo "$1 failed"; tail -5 $OUT/b.err; return 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b.json').readline()); print('arm [$1]', d['value'], d['ms_per_step'], d['config'].get('request_streams'), d['config'].get('lanes_per_stream'))"
}
for rep in 1 2 3; do
  run "" || exit 1
  run "--split 8" || exit 1
  run "--split 4 --lanes 2" || exit 1
done
