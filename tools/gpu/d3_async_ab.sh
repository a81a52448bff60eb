# dwpw3 hand-off A/B: unit tests of the async build (LDS counters), then timings of both builds (two rounds)
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/d3as}
mkdir -p "$OUT"
MLIC_HIP_LIB=$PWD/mlic_amd/libmlic_hip_as.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_conv.py -m gpu -x -v \
  --timeout 120 --timeout-method thread -k "dwpw" > "$OUT/unit.log" 2>&1
rc=$?; tail -2 "$OUT/unit.log"; [ $rc -eq 0 ] || { grep -E "^FAILED|^E  " "$OUT/unit.log" | head -20; exit $rc; }
for r in 1 2; do
  timeout -k 10 120 python3 -u tools/gpu/dwpw_ab.py barrier >> "$OUT/time.log" 2>&1 || { tail -5 "$OUT/time.log"; exit 1; }
  MLIC_HIP_LIB=$PWD/mlic_amd/libmlic_hip_as.so timeout -k 10 120 python3 -u tools/gpu/dwpw_ab.py async >> "$OUT/time.log" 2>&1 || { tail -5 "$OUT/time.log"; exit 1; }
done
grep epi "$OUT/time.log"
