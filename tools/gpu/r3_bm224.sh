cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/bm224}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 180 python3 -u tools/gpu/bench_conv.py 8 640 224 68 120 1 1 1  8 384 224 68 120 1 1 1  8 224 224 68 120 1 1 0 2>&1 | grep -v amdgpu.ids | tee "$OUT/conv.log" || exit 1
bash tools/gpu/r3_quick.sh "$OUT" "x4" || exit 1
