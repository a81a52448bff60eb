# request-stream split A/B on the main config (timed steps only)
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/split; mkdir -p $OUT
run() { tag=$1; shift; timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag failed $?"; tail -5 $OUT/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/$tag.json').readline()); print('$tag', d['value'], d['ms_per_step'], d['wall_ms_per_step'], d['host_thread_ms_per_step'])"; }
run base
run s4l1 --split 4 --lanes 1
run s2l2 --split 2 --lanes 2
run s4l2 --split 4 --lanes 2
run s8l1 --split 8 --lanes 1 --group-concurrency 8
run base2
