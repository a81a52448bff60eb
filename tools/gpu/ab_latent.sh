# latent-resolution GEMM variants (x3v2 256x256 / 128x128, x4): usage bash tools/gpu/ab_latent.sh <outdir>
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/ab}
mkdir -p "$OUT"
S="8 640 224 68 120 1 1 1  8 480 224 68 120 1 1 1  8 352 224 68 120 1 1 1  8 288 288 68 120 1 1 0  8 192 192 68 120 1 1 0  8 320 1280 17 30 3 1 129"
for v in "MLIC_BENCH_IMPL=2" "MLIC_BENCH_IMPL=2 MLIC_V2_WIDE=0" "MLIC_BENCH_IMPL=7" "MLIC_BENCH_IMPL=6"; do
  echo "== $v"
  env $v timeout -k 10 120 python3 -u tools/gpu/bench_conv.py $S 2>&1 | grep -v amdgpu.ids || { echo "failed $v"; exit 1; }
done
