# dwpw3 packed-fp32 A/B: unit tests on the default build, then the timing of each arm (two rounds)
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/d3pk}
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_conv.py -m gpu -x -v --timeout 120 --timeout-method thread -k "dwpw" > "$OUT/unit.log" 2>&1
rc=$?; tail -2 "$OUT/unit.log"; [ $rc -eq 0 ] || { grep -E "^FAILED|^E  " "$OUT/unit.log" | head -20; exit $rc; }
for r in 1 2; do
  for arm in p11 tpf p00 p10 p01; do
    lib=mlic_amd/libmlic_hip_$arm.so; [ $arm = p11 ] && lib=mlic_amd/libmlic_hip.so
    MLIC_HIP_LIB=$PWD/$lib timeout -k 10 120 python3 -u tools/gpu/dwpw_ab.py $arm >> "$OUT/time.log" 2>&1 || { tail -5 "$OUT/time.log"; exit 1; }
  done
done
grep epi "$OUT/time.log"
