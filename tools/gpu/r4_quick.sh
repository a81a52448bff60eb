# quick check: the tests touching a change (-k filter), then the default bench line + per-layer table
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/quick}
K=${2:-"linear_attention or local_attention or module_vectors or roundtrip"}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" \
  > "$OUT/tests.log" 2>&1 || { echo "tests failed $?"; tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
timeout -k 10 600 python3 -u bench.py --no-cpu-baseline --layers-out "$OUT/layers.tsv" > "$OUT/bench.json" \
  2> "$OUT/bench.err" || { echo "bench failed $?"; tail -30 "$OUT/bench.err"; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']
print('value', d['value'], 'ms/step', d['ms_per_step'], 'iso total', d['gpu_kernel_ms_isolated_share'])
print('frac', r['frac'], 'step_frac', r['step_frac']); print(d['kernel_families_ms_isolated_share'])"
