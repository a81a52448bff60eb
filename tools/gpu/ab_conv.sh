# Conv-layer A/B on the GPU box: each variant is an environment assignment list (MLIC_BENCH_IMPL
# forces a kernel family, the MLIC_X4_* / MLIC_V2_* switches select variants); the shapes are
# "B Cin Cout H W K stride epi" groups for tools/gpu/bench_conv.py.  Examples used in round 2:
#   bash tools/gpu/ab_conv.sh "8 192 768 272 480 3 1 128  8 640 6400 68 120 1 1 0" "MLIC_BENCH_IMPL=7" "MLIC_BENCH_IMPL=8"
#   bash tools/gpu/ab_conv.sh "16 224 128 32 48 1 1 1  16 640 224 32 48 1 1 1" "MLIC_BENCH_IMPL=2" "MLIC_BENCH_IMPL=3" "MLIC_BENCH_IMPL=7"
cd "$GRAFT_REPO_ROOT"
S=$1
shift
for v in "$@"; do
  echo "== $v"
  env $v timeout -k 10 120 python3 -u tools/gpu/bench_conv.py $S 2>&1 | grep -v amdgpu.ids || { echo "failed: $v"; exit 1; }
done
