# conv-epilogue GELU: library erff (default) vs the chain kernel's branch-free form (A/B library)
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/gelu}
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2; do
for lib in mlic_amd/libmlic_hip.so tools/gpu/libmlic_gelufast.so; do
MLIC_HIP_LIB=$PWD/$lib timeout -k 10 180 python3 -u tools/gpu/bench_conv.py 8 192 768 272 480 3 1 129  8 192 768 272 480 3 1 128  8 192 768 136 240 3 1 129 2>&1 | grep -v amdgpu.ids | sed "s|^|$(basename $lib) |" | tee -a "$OUT/conv.log" || exit 1
done
done
