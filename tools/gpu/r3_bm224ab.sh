cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/bm224ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2; do
for v in 1 0; do
MLIC_X4_BM224=$v timeout -k 10 180 python3 -u tools/gpu/bench_conv.py 8 640 224 68 120 1 1 1  8 384 224 68 120 1 1 1  8 224 224 68 120 1 1 0  8 448 224 68 120 3 1 0 2>&1 | grep -v amdgpu.ids | sed "s/^/bm224=$v /" | tee -a "$OUT/conv.log" || exit 1
done
done
