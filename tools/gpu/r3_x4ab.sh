# x4 scheduling experiments (MLIC_X4_ABL bits 16 / 32 / 64) on the heaviest x4 shapes, plus the conv
# tests under the chosen bits.   bash tools/gpu/r3_x4ab.sh <outdir> "<abl values>"
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/x4ab}; VALS=${2:-0 16 32 64 80}
mkdir -p "$OUT"
export TMPDIR=/tmp
S="8 192 768 272 480 3 1 128  8 192 768 136 240 3 1 128  8 640 6400 68 120 1 1 0  8 480 1920 17 30 3 1 128"
for v in $VALS; do
  echo "== abl $v" | tee -a "$OUT/x4ab.log"
  MLIC_X4_ABL=$v timeout -k 10 180 python3 -u tools/gpu/bench_conv.py $S 2>&1 | grep -v amdgpu.ids | tee -a "$OUT/x4ab.log" || { echo "failed: $v"; exit 1; }
done
for v in $VALS; do
  MLIC_X4_ABL=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 120 --timeout-method thread -k "x4" > "$OUT/t.log" 2>&1 || { echo "x4 tests failed abl $v"; tail -20 "$OUT/t.log"; exit 1; }
  echo "abl $v tests: $(tail -1 "$OUT/t.log")"
done
