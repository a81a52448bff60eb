# x4 step order A/B: the product library (fragment reads first, staging after the first pixel group's
# MFMAs) against libmlic_hip_x4sf.so (make EXTRA=-DMLIC_X4_STAGING_FIRST: the round-3 order)
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/x4early}
mkdir -p "$OUT"
export TMPDIR=/tmp
for lib in libmlic_hip_x4sf.so libmlic_hip.so; do
  MLIC_HIP_LIB=$PWD/mlic_amd/$lib timeout -k 10 200 python3 -u tools/gpu/bench_conv.py > "$OUT/bench_$lib.log" 2>&1 ||
    { echo "bench $lib failed $?"; tail -20 "$OUT/bench_$lib.log"; exit 1; }
  echo "$lib"; grep impl "$OUT/bench_$lib.log"
done
