# r3_configs.sh without the exact-fp32 line (unchanged by x4 changes): per-config lines + 8-rank emulation
# multi-job configs, and the exact-fp32 MFMA (--precision 0) line.   bash tools/gpu/r3_configs.sh <outdir>
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/configs}
mkdir -p "$OUT"
export TMPDIR=/tmp
CONFIGS="${CONFIGS:-kodak s1080 sd1080 vbr-mixed kodak-sweep}" bash tools/gpu/record_configs.sh "$OUT" || exit 1
for c in kodak-sweep vbr-mixed; do
  timeout -k 10 400 python3 -u bench.py --config "$c" --emulate-world 8 --emulate-rank 0 --no-cpu-baseline \
    > "$OUT/bench_${c}_emu8r0.json" 2> "$OUT/bench_${c}_emu8r0.err" || { echo "emu $c failed $?"; tail -20 "$OUT/bench_${c}_emu8r0.err"; exit 1; }
  echo "emu8 $c: $(head -c 300 "$OUT/bench_${c}_emu8r0.json")"
done
