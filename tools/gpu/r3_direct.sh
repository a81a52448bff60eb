# x4 1x1 direct-B gate: conv tests (x4), parity subset, bench + layers; then the same bench with the
# packed path (MLIC_X4_DIRECT=0) and the 224-row tile off (MLIC_X4_BM224=0) for the A/B
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/direct}
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu/r3_quick.sh "$OUT" "x4 or split_operand" || exit 1
MLIC_X4_DIRECT=0 timeout -k 10 600 python -u bench.py --no-cpu-baseline --layers-out "$OUT/layers_packed.tsv" > "$OUT/bench_packed.json" 2> "$OUT/bench_packed.err" || exit 1
head -c 200 "$OUT/bench_packed.json"; echo
MLIC_X4_BM224=0 timeout -k 10 600 python -u bench.py --no-cpu-baseline --layers-out "$OUT/layers_no224.tsv" > "$OUT/bench_no224.json" 2> "$OUT/bench_no224.err" || exit 1
head -c 200 "$OUT/bench_no224.json"; echo
