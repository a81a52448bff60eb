# kernel trace of the timed configuration (no profiled passes), kept for the occupancy analysis
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/busy; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o run -- \
  python3 -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-roofline > $OUT/bench.json 2> $OUT/bench.err || { echo fail $?; tail $OUT/bench.err; exit 1; }
f=$(ls $OUT/tr/*kernel_trace.csv $OUT/tr/*/*kernel_trace.csv 2>/dev/null | head -1); echo $f
python3 tools/trace_busy.py $f 0.2 && python3 tools/trace_busy.py $f 0.0
gzip -c $f > $OUT/kernel_trace.csv.gz; rm -rf $OUT/tr; cat $OUT/bench.json | head -c 300
