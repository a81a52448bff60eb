# Round-5 check: dwpw ablation sweep, the coder / interop parity tests, and short bench lines (enc+dec and
# decode-only).  usage: bash tools/gpu/r5_check.sh <outdir> [stages]   stages: abl tests bench
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/r5}
STAGES=${2:-"abl tests bench"}
mkdir -p "$OUT"
has() { case " $STAGES " in *" $1 "*) return 0;; esac; return 1; }
if has abl; then
  for N in base $ABL; do
    if [ "$N" = base ]; then LIBV=""; else LIBV=$PWD/mlic_amd/libmlic_hip_dp$N.so; fi
    env ${LIBV:+MLIC_HIP_LIB=$LIBV} timeout -k 10 120 python3 -u tools/gpu/dwpw_ab.py dp$N >> "$OUT/abl.log" 2>&1 || { echo "abl $N failed"; tail -5 "$OUT/abl.log"; exit 1; }
  done
  cat "$OUT/abl.log" | grep epi
fi
if has tests; then
  MLIC_PARITY_OUT="$OUT/parity_counts.json" timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 \
    --timeout-method thread -k "${TESTK:-roundtrip or streams or interop or batched_y or lanes or file_format}" > "$OUT/tests.log" 2>&1
  rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || { grep -E "^FAILED|^E  " "$OUT/tests.log" | head -30; exit $rc; }
fi
if has bench; then
  timeout -k 10 400 python3 -u bench.py --steps 3 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
  head -c 600 "$OUT/bench.json"; echo
  timeout -k 10 400 python3 -u bench.py --steps 3 --phase decode > "$OUT/bench_decode.json" 2> "$OUT/bench_decode.err" || { echo "bench decode failed"; tail -20 "$OUT/bench_decode.err"; exit 1; }
  head -c 600 "$OUT/bench_decode.json"; echo
fi
echo "r5_check done"
