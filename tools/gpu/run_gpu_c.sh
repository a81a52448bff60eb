cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 2 --profile-lanes 1 --layers-out gpurun_out/layers_iso.tsv > gpurun_out/bench_iso.json 2> gpurun_out/bench_iso.err || { echo "bench failed $?"; tail -30 gpurun_out/bench_iso.err; exit 1; }
cat gpurun_out/bench_iso.json
