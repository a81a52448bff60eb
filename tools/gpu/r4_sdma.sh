# copy engine A/B: are host<->device copies blit kernels (copyBuffer) by default, and does SDMA change the step?
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/sdma; mkdir -p $OUT; export TMPDIR=/tmp
env | grep -i -E "sdma|blit|HSA_|ROC_|GPU_|HIP_" | sort > $OUT/env.txt; cat $OUT/env.txt
run() { tag=$1; shift; timeout -k 10 300 "$@" python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --split 4 --lanes 2 > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag failed $?"; tail -5 $OUT/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/$tag.json').readline()); print('$tag', d['value'], d['ms_per_step'], d['host_thread_ms_per_step'])"; }
run def env && run sdma1 env HSA_ENABLE_SDMA=1 && run sdma0 env HSA_ENABLE_SDMA=0 && run def2 env
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p1 -o run -- python3 -u bench.py --lanes 1 --batch 8 --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > /dev/null 2>&1 || echo prof1 fail
grep -i copy $OUT/p1/*kernel_stats.csv $OUT/p1/*/*kernel_stats.csv 2>/dev/null | head -5
