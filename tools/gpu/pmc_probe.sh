# PMC counter passes over one conv-layer micro-benchmark (tools/gpu/bench_conv.py), one rocprofv3
# run per pass; prints per-kernel means.  usage on the box:
#   bash tools/gpu/pmc_probe.sh <outdir> <kernel-substring> "<B Cin Cout H W K s epi>" "<pass1 counters>" ["<pass2>" ...]
cd "$GRAFT_REPO_ROOT"
OUT=$1; KERN=$2; SHAPE=$3; shift 3
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for pass in "$@"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $pass -d "$OUT/p$i" -o run -- python3 -u tools/gpu/bench_conv.py $SHAPE \
    > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed $?"; tail -5 "$OUT/p$i.log"; exit 1; }
  db=$(find "$OUT/p$i" -name '*.db' | head -n 1)
  python3 tools/pmc_summary.py "$db" "$KERN"
done
