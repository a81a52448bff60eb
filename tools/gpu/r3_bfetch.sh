# x4 bound: the K=3 / K=5 loops with B fetched every tap (default) vs once per chunk (MLIC_X4_ABL=16,
# diagnostics: wrong results)
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/bfetch}
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2; do
for a in 0 16; do
MLIC_X4_ABL=$a timeout -k 10 180 python3 -u tools/gpu/bench_conv.py 8 192 768 272 480 3 1 128  8 192 768 136 240 3 1 128  8 224 96 68 120 5 1 0  8 192 192 544 960 3 1 0 2>&1 | grep -v amdgpu.ids | sed "s|^|abl=$a |" | tee -a "$OUT/conv.log" || exit 1
done
done
