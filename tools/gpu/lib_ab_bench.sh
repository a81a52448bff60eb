# whole-model A/B between library builds: the isolated pass (one lane, 8 images) and the default line per
# build, alternating two rounds.  usage: bash tools/gpu/lib_ab_bench.sh <outdir> tag1 tag2 ... (mlic_amd/libmlic_hip_<tag>.so)
cd "$GRAFT_REPO_ROOT"
OUT=$1; shift
mkdir -p "$OUT"
for r in 1 2; do
  for t in "$@"; do
    MLIC_HIP_LIB=$PWD/mlic_amd/libmlic_hip_$t.so timeout -k 10 400 python3 -u bench.py --steps 3 --no-cpu-baseline \
      > "$OUT/bench_${t}_$r.json" 2> "$OUT/bench_${t}_$r.err" || { echo "bench $t failed"; tail -5 "$OUT/bench_${t}_$r.err"; exit 1; }
    python3 -c "import json,sys; b=json.load(open(sys.argv[1])); print(sys.argv[2], b['value'], 'chain iso ms', b['kernel_families_ms_isolated_share'].get('chain_kernel'), 'frac', [x['frac'] for x in b['roofline']['runners_up'] if x['kernel']=='chain_kernel'])" "$OUT/bench_${t}_$r.json" $t
  done
done
