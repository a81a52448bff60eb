# round 6: x4 tile height at the latent grid: LRP's first 1x1 (-> 224, GELU) and h_s's 480 -> 640, isolated, alternating
cd "$GRAFT_REPO_ROOT"
SH="8 480 224 68 120 1 1 1 8 640 224 68 120 1 1 1 8 480 640 68 120 1 1 0"
for rep in 1 2; do
  for arm in "" "224:256,640:192" "224:128,640:256"; do
    echo "== [$arm]"
    MLIC_X4_BM_FOR="$arm" timeout -k 10 120 python3 tools/gpu/bench_conv.py $SH || exit 1
  done
done
