# end-of-round check: the whole GPU suite (no -x; parity counts), then smoke()
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/final}
mkdir -p "$OUT"
export TMPDIR=/tmp
MLIC_PARITY_OUT="$OUT/parity_counts.json" timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 \
  --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?
tail -1 "$OUT/gpu_tests.log"
grep -E "^FAILED|AssertionError" "$OUT/gpu_tests.log" | head -10
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed $?"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
