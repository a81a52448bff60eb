# dwpw2 (producer / consumer fused depthwise + pointwise) bring-up: kernel tests, timing against the
# one-wave-per-SIMD kernel (MLIC_DWPW2=0), model parity that runs it, a bench line.
#   bash tools/gpu/dwpw2_check.sh <outdir> [stages]   stages: unit time model bench
#   D2FORM=1|2 (default 2): the form the unit / model / bench stages select (MLIC_DWPW2)
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/d2}
STAGES=${2:-"unit time model bench"}
F=${D2FORM:-2}
mkdir -p "$OUT"
has() { case " $STAGES " in *" $1 "*) return 0;; esac; return 1; }
if has unit; then
  MLIC_DWPW2=$F timeout -k 10 300 python3 -u -m pytest tests/test_gpu_conv.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -k "dwpw" > "$OUT/unit.log" 2>&1
  rc=$?; tail -3 "$OUT/unit.log"; [ $rc -eq 0 ] || { grep -E "^FAILED|^E  " "$OUT/unit.log" | head -30; exit $rc; }
fi
if has time; then
  MLIC_DWPW2=0 timeout -k 10 120 python3 -u tools/gpu/dwpw_ab.py v1 > "$OUT/time.log" 2>&1 || { tail -5 "$OUT/time.log"; exit 1; }
  MLIC_DWPW2=1 timeout -k 10 120 python3 -u tools/gpu/dwpw_ab.py v2 >> "$OUT/time.log" 2>&1 || { tail -5 "$OUT/time.log"; exit 1; }
  MLIC_DWPW2=2 timeout -k 10 120 python3 -u tools/gpu/dwpw_ab.py v3 >> "$OUT/time.log" 2>&1 || { tail -5 "$OUT/time.log"; exit 1; }
  MLIC_DWPW2=0 timeout -k 10 120 python3 -u tools/gpu/dwpw_ab.py v1 >> "$OUT/time.log" 2>&1 || { tail -5 "$OUT/time.log"; exit 1; }
  grep epi "$OUT/time.log"
fi
if has model; then
  MLIC_DWPW2=$F MLIC_PARITY_OUT="$OUT/parity_counts.json" timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v \
    --timeout 300 --timeout-method thread -k "${TESTK:-fixture or 1080p or roundtrip or kodak or module_vectors}" > "$OUT/model.log" 2>&1
  rc=$?; tail -3 "$OUT/model.log"; [ $rc -eq 0 ] || { grep -E "^FAILED|^E  " "$OUT/model.log" | head -30; exit $rc; }
fi
if has bench; then
  MLIC_DWPW2=$F timeout -k 10 400 python3 -u bench.py --steps 3 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
  head -c 300 "$OUT/bench.json"; echo
fi
echo "dwpw2_check done"
