# 96-row x4 tile: conv tests, the reprojection shapes, the parity gate and the main line
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/bm96}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 180 python3 -u tools/gpu/bench_conv.py 8 288 96 68 120 5 1 0  8 128 96 68 120 5 1 0  8 96 96 68 120 3 1 1 2>&1 | grep -v amdgpu.ids | tee "$OUT/conv.log" || exit 1
bash tools/gpu/r3_quick.sh "$OUT" "x4" || exit 1
