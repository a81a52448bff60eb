# round 6: x4 tile height for h_s's 3x3 convs (480 -> 1920 at 34 x 60, 320 -> 1280 at 17 x 30), isolated, alternating
cd "$GRAFT_REPO_ROOT"
SH="8 480 1920 34 60 3 1 129 8 320 1280 17 30 3 1 129"
for rep in 1 2; do
  for arm in "" "1920:128,1280:128" "1920:192,1280:192" "1280:64"; do
    echo "== [$arm]"
    MLIC_X4_BM_FOR="$arm" timeout -k 10 120 python3 tools/gpu/bench_conv.py $SH || exit 1
  done
done
