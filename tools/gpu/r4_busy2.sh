# default bench line (split 4 x 2 lanes) + kernel trace of the timed configuration for the occupancy analysis
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/busy2; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench fail $?; tail $OUT/bench.err; exit 1; }
head -c 600 $OUT/bench.json; echo
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o run -- \
  python3 -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-roofline > $OUT/bench_tr.json 2> $OUT/bench_tr.err || { echo fail $?; tail $OUT/bench_tr.err; exit 1; }
f=$(ls $OUT/tr/*kernel_trace.csv $OUT/tr/*/*kernel_trace.csv 2>/dev/null | head -1)
gzip -c $f > $OUT/kernel_trace.csv.gz; rm -rf $OUT/tr; head -c 300 $OUT/bench_tr.json
