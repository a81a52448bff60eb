# 8-rank emulation (rank 0 of 8: its job share, 1/8 of the host cores) of the two multi-job configs, and
# the exact-fp32 MFMA (--precision 0) line.   bash tools/gpu/r3_emu.sh <outdir>
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/emu}
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in kodak-sweep vbr-mixed; do
  timeout -k 10 400 python3 -u bench.py --config "$c" --emulate-world 8 --emulate-rank 0 --no-cpu-baseline \
    > "$OUT/bench_${c}_emu8r0.json" 2> "$OUT/bench_${c}_emu8r0.err" || { echo "emu $c failed $?"; tail -20 "$OUT/bench_${c}_emu8r0.err"; exit 1; }
  echo "emu8 $c: $(head -c 300 "$OUT/bench_${c}_emu8r0.json")"
done
timeout -k 10 900 python3 -u bench.py --precision 0 --no-cpu-baseline --layers-out "$OUT/layers_prec0.tsv" \
  > "$OUT/bench_prec0.json" 2> "$OUT/bench_prec0.err" || { echo "prec0 failed $?"; tail -20 "$OUT/bench_prec0.err"; exit 1; }
echo "prec0: $(head -c 300 "$OUT/bench_prec0.json")"
