# dwpw3 timing probes against the default build (two rounds): $@ = library tags (mlic_amd/libmlic_hip_<tag>.so)
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/d3probe
mkdir -p "$OUT"
for r in 1 2; do
  timeout -k 10 120 python3 -u tools/gpu/dwpw_ab.py default >> "$OUT/time.log" 2>&1 || { tail -5 "$OUT/time.log"; exit 1; }
  for t in "$@"; do
    MLIC_HIP_LIB=$PWD/mlic_amd/libmlic_hip_$t.so timeout -k 10 120 python3 -u tools/gpu/dwpw_ab.py $t >> "$OUT/time.log" 2>&1 || { tail -5 "$OUT/time.log"; exit 1; }
  done
done
grep epi "$OUT/time.log"
