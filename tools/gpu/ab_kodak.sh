# Kodak-size (768x512: latent 32x48) conv variants + the kodak config's layer table; usage: bash tools/gpu/ab_kodak.sh <out>
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/kodak}
mkdir -p "$OUT"
S="16 640 224 32 48 1 1 1  16 480 224 32 48 1 1 1  16 352 224 32 48 1 1 1  16 288 288 32 48 1 1 0  16 640 6400 32 48 1 1 0  16 288 96 32 48 5 1 0"
for v in "MLIC_BENCH_IMPL=2" "MLIC_BENCH_IMPL=7"; do
  echo "== $v"
  env $v timeout -k 10 120 python3 -u tools/gpu/bench_conv.py $S 2>&1 | grep -v amdgpu.ids || { echo "failed $v"; exit 1; }
done
timeout -k 10 300 python3 -u bench.py --config kodak --no-cpu-baseline --layers-out "$OUT/layers_kodak.tsv" > "$OUT/bench_kodak.json" 2> "$OUT/err" || { echo "bench failed"; tail -5 "$OUT/err"; exit 1; }
head -c 200 "$OUT/bench_kodak.json"
