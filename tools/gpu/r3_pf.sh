# x4 direct 1x1: load lookahead 1 vs 2 K-steps (MLIC_X4_PF), conv tests for x4
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/pf}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 120 --timeout-method thread -k "x4" > "$OUT/conv_tests.log" 2>&1 || { echo "conv tests failed $?"; tail -30 "$OUT/conv_tests.log"; exit 1; }
tail -1 "$OUT/conv_tests.log"
for r in 1 2; do
for pf in 1 2; do
MLIC_X4_PF=$pf timeout -k 10 180 python3 -u tools/gpu/bench_conv.py 8 288 288 68 120 1 1 0  8 480 640 68 120 1 1 0  8 960 320 68 120 1 1 0  8 352 192 68 120 1 1 1  8 256 96 68 120 1 1 0 2>&1 | grep -v amdgpu.ids | sed "s/^/pf=$pf /" | tee -a "$OUT/conv.log" || exit 1
done
done
