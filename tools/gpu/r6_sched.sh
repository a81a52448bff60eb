# round 6: per-step join vs back-to-back request streams (bench.py --schedule), alternating on one box
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6sc; mkdir -p $OUT
for rep in 1 2 3; do
  for sch in join streams; do
    timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --no-decode-record \
      --schedule $sch > $OUT/b.json 2> $OUT/b.err || { echo "$sch failed"; tail -5 $OUT/b.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/b.json').readline()); print('$sch', d['value'], d['ms_per_step'])"
  done
done
