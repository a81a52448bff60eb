# x4 step order A/B (MLIC_X4_ABL=16: staging before the step's fragment reads, round-3 order)
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/x4early}
mkdir -p "$OUT"
export TMPDIR=/tmp
for a in 16 0; do
  MLIC_X4_ABL=$a timeout -k 10 200 python3 -u tools/gpu/bench_conv.py > "$OUT/bench_abl$a.log" 2>&1 ||
    { echo "bench abl=$a failed $?"; tail -20 "$OUT/bench_abl$a.log"; exit 1; }
  echo "abl=$a"; grep impl "$OUT/bench_abl$a.log"
done
