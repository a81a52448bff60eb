# GPU suite + dwpw data microbench + bench (default and 4 request streams x 2 lanes)
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/tail; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "^FAILED|^E  " $OUT/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 240 python3 -u tools/gpu/dwpw_data.py > $OUT/dwpw_data.log 2>&1 || { echo dd fail; exit 1; }
grep -v amdgpu.ids $OUT/dwpw_data.log
run() { tag=$1; shift; timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag failed $?"; tail -5 $OUT/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/$tag.json').readline()); print('$tag', d['value'], d['ms_per_step'], d['host_thread_ms_per_step'])"; }
run base && run s4l2 --split 4 --lanes 2 && run l8 --lanes 8 && run base2
