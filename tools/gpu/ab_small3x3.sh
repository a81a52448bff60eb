cd "$GRAFT_REPO_ROOT"
S="8 320 1280 8 12 3 1 129  8 480 1920 16 24 3 1 129  8 320 1280 17 30 3 1 129  8 256 256 68 120 1 1 0  8 224 224 68 120 1 1 0  8 256 256 32 48 1 1 0"
for v in "MLIC_BENCH_IMPL=2" "MLIC_BENCH_IMPL=7" "MLIC_BENCH_IMPL=6"; do
  echo "== $v"
  env $v timeout -k 10 120 python3 -u tools/gpu/bench_conv.py $S 2>&1 | grep -v amdgpu.ids || { echo "failed $v"; exit 1; }
done
