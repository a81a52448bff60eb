# fused dwpw bit-exactness test + micro-benchmark only.   bash tools/gpu/r3_dwpw_quick.sh <outdir>
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/dwpwq}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -v --timeout 120 --timeout-method thread -k dwpw > "$OUT/dwpw_test.log" 2>&1 || { echo "dwpw test failed $?"; tail -40 "$OUT/dwpw_test.log"; exit 1; }
tail -2 "$OUT/dwpw_test.log"
for shp in "8 192 544 960" "8 192 272 480" "8 192 136 240" "8 192 68 120" "8 96 544 960" "8 48 1088 1920"; do
  timeout -k 10 120 python -u tools/gpu/bench_dwpw.py $shp 2>&1 | grep -v amdgpu.ids >> "$OUT/bench_dwpw.log" || { echo "bench_dwpw failed"; tail -20 "$OUT/bench_dwpw.log"; exit 1; }
done
cat "$OUT/bench_dwpw.log"
