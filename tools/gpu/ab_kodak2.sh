# Kodak-size latent 1x1 convs: x3v2 / pw_resident / x4 (16 images, 32 x 48); usage: bash tools/gpu/ab_kodak2.sh
cd "$GRAFT_REPO_ROOT"
S="16 224 128 32 48 1 1 1  16 192 128 32 48 1 1 1  16 128 32 32 48 1 1 88  16 96 192 32 48 1 1 1  16 128 128 32 48 1 1 0  16 64 64 32 48 1 1 0  16 32 96 32 48 1 1 0  16 96 128 32 48 1 1 1  16 128 64 32 48 1 1 64  16 192 192 32 48 1 1 0  16 192 320 8 12 1 1 0  16 640 224 32 48 1 1 1"
for v in 2 3 7; do
  echo "== impl $v"
  MLIC_BENCH_IMPL=$v timeout -k 10 120 python3 -u tools/gpu/bench_conv.py $S 2>&1 | grep -v amdgpu.ids
done
exit 0
