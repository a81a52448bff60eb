# config experiments: sweep / VBR with more concurrent groups, fewer lanes; the small-decoder layer
# table.   bash tools/gpu/r3_cfgexp.sh <outdir>
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/cfgexp}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --no-roofline "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed $?"; tail -20 "$OUT/$n.err"; exit 1; }
  python3 -c "import json,sys; b=json.loads(open('$OUT/$n.json').readline()); print('$n', b['value'], b['ms_per_step'], b.get('batches_per_step'), b.get('group_concurrency'), b.get('lanes'))"
}
run sweep_gc6 --config kodak-sweep --group-concurrency 6
run sweep_gc12_l2 --config kodak-sweep --group-concurrency 12 --lanes 2
run sweep_gc6_l2 --config kodak-sweep --group-concurrency 6 --lanes 2
run sweep_emu_l2 --config kodak-sweep --emulate-world 8 --emulate-rank 0 --lanes 2
run sweep_emu_l6 --config kodak-sweep --emulate-world 8 --emulate-rank 0 --lanes 6
run vbr_l6 --config vbr-mixed --lanes 6
run vbr_l2_gc2 --config vbr-mixed --lanes 2
timeout -k 10 400 python3 -u bench.py --config sd1080 --no-cpu-baseline --layers-out "$OUT/layers_sd1080.tsv" > "$OUT/sd1080.json" 2> "$OUT/sd1080.err" || { echo "sd failed"; tail -20 "$OUT/sd1080.err"; exit 1; }
echo "sd1080 $(head -c 200 "$OUT/sd1080.json")"
