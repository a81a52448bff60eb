# pixel-pair dwpw / pw2 checks: dwpw tests, conv tests with MLIC_PW2=1, micro-bench with and without
# MLIC_PW2, then the default bench line with MLIC_DWPW=1 [+ MLIC_PW2=1].   bash tools/gpu/r3_pw2.sh <outdir>
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/pw2}
mkdir -p "$OUT"
export TMPDIR=/tmp
MLIC_PW2=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/conv_test_pw2.log" 2>&1 || { echo "conv tests (pw2) failed $?"; tail -40 "$OUT/conv_test_pw2.log"; exit 1; }
tail -1 "$OUT/conv_test_pw2.log"
for shp in "8 192 544 960" "8 192 272 480" "8 128 544 960"; do
  for e in 0 1; do
    MLIC_PW2=$e timeout -k 10 120 python -u tools/gpu/bench_dwpw.py $shp > "$OUT/b.tmp" 2>&1 || { echo "bench failed"; cat "$OUT/b.tmp"; exit 1; }
    echo "pw2=$e $(grep fused "$OUT/b.tmp")" | tee -a "$OUT/micro.log"
  done
done
MLIC_DWPW=1 timeout -k 10 600 python -u bench.py --no-cpu-baseline --layers-out "$OUT/layers_dwpw.tsv" > "$OUT/bench_dwpw.json" 2> "$OUT/bench_dwpw.err" || { echo "bench failed"; tail -20 "$OUT/bench_dwpw.err"; exit 1; }
head -c 300 "$OUT/bench_dwpw.json"; echo
MLIC_DWPW=1 MLIC_PW2=1 timeout -k 10 600 python -u bench.py --no-cpu-baseline --layers-out "$OUT/layers_dwpw_pw2.tsv" > "$OUT/bench_dwpw_pw2.json" 2> "$OUT/bench_dwpw_pw2.err" || { echo "bench failed"; tail -20 "$OUT/bench_dwpw_pw2.err"; exit 1; }
head -c 300 "$OUT/bench_dwpw_pw2.json"; echo
