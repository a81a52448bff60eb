# 192-row x4 tile: conv tests, the SD dense conv shapes, the parity gate, the main and SD lines
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/bm192}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 180 python3 -u tools/gpu/bench_conv.py 8 192 192 544 960 3 1 1  8 192 192 544 960 3 2 1  8 96 160 272 480 3 1 0 2>&1 | grep -v amdgpu.ids | tee "$OUT/conv.log" || exit 1
bash tools/gpu/r3_quick.sh "$OUT" "x4 or dwpw or pw_resident" || exit 1
timeout -k 10 400 python3 -u bench.py --config sd1080 --no-cpu-baseline --layers-out "$OUT/layers_sd1080.tsv" > "$OUT/sd1080.json" 2> "$OUT/sd1080.err" || { echo "sd failed"; tail -20 "$OUT/sd1080.err"; exit 1; }
echo "sd1080 $(head -c 200 "$OUT/sd1080.json")"
