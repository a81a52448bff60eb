# LocalContext attention A/B between library builds: the local-attention GPU tests on the current
# library, then the default line per build, alternating two rounds, with the isolated pass's
# local_attn_kernel time.  usage: bash tools/gpu/la_ab.sh <outdir> tag1 tag2 ... (mlic_amd/libmlic_hip_<tag>.so)
cd "$GRAFT_REPO_ROOT"
OUT=$1; shift
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_conv.py tests/test_gpu_parity.py -m gpu -k "local" -v --timeout 120 \
  --timeout-method thread > "$OUT/la_tests.log" 2>&1 || { echo "tests failed $?"; tail -30 "$OUT/la_tests.log"; exit 1; }
tail -1 "$OUT/la_tests.log"
for r in 1 2; do
  for t in "$@"; do
    MLIC_HIP_LIB=$PWD/mlic_amd/libmlic_hip_$t.so timeout -k 10 400 python3 -u bench.py --steps 3 --no-cpu-baseline \
      --layers-out "$OUT/layers_${t}_$r.tsv" > "$OUT/bench_${t}_$r.json" 2> "$OUT/bench_${t}_$r.err" ||
      { echo "bench $t failed"; tail -5 "$OUT/bench_${t}_$r.err"; exit 1; }
    python3 -c "
import json, sys
b = json.load(open(sys.argv[1]))
la = [float(l.split('\t')[4]) for l in open(sys.argv[3]) if l.split('\t')[2] == 'local_attn_kernel']
print(sys.argv[2], b['value'], 'local_attn calls', len(la), 'ms/call', round(sum(la) / max(len(la), 1), 4))
" "$OUT/bench_${t}_$r.json" $t "$OUT/layers_${t}_$r.tsv"
  done
done
