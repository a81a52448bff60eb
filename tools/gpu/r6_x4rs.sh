# round 6: x4 operand staging A/B on the 3x3 shapes: register staging (default) vs LDS-DMA (MLIC_X4_RS=0) vs
# halo-staged B for 3x3 (MLIC_X4_HALO=2), alternating, one box
cd "$GRAFT_REPO_ROOT"
SH="8 192 768 272 480 3 1 129 8 192 768 136 240 3 1 128 8 480 1920 34 60 3 1 129 8 320 1280 17 30 3 1 129"
for rep in 1 2 3; do
for v in def rs0 h3; do
  unset MLIC_X4_RS MLIC_X4_HALO
  [ $v = rs0 ] && export MLIC_X4_RS=0
  [ $v = h3 ] && export MLIC_X4_HALO=2
  echo "== $v rep $rep"
  timeout -k 10 120 python3 tools/gpu/bench_conv.py $SH || exit 1
done; done
