# round 6: x4 register-staged loop decomposition (diagnostics libraries built with -DMLIC_X4_ABL_RS=mask)
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6x; mkdir -p $OUT
SH="8 192 768 272 480 3 1 129 8 192 768 136 240 3 1 128 8 288 96 68 120 5 1 0 8 640 224 68 120 1 1 1"
for rep in 1 2; do
for v in "" 1 2 4 3; do
  if [ -n "$v" ]; then export MLIC_HIP_LIB=$PWD/mlic_amd/libmlic_hip_x4abl$v.so; else unset MLIC_HIP_LIB; fi
  echo "== abl=${v:-0} rep $rep"
  timeout -k 10 120 python3 tools/gpu/bench_conv.py $SH || exit 1
done; done
