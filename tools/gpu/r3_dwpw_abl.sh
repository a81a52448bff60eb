# fused dwpw (pixel-pair form) ablation timings + PMC passes.   bash tools/gpu/r3_dwpw_abl.sh <outdir>
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/dwpw_abl}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 120 --timeout-method thread -k dwpw > "$OUT/dwpw_test.log" 2>&1 || { echo "dwpw test failed $?"; tail -40 "$OUT/dwpw_test.log"; exit 1; }
tail -1 "$OUT/dwpw_test.log"
for v in base abl1 abl2 abl4; do
  if [ $v = base ]; then L=mlic_amd/libmlic_hip.so; else L=tools/gpu/var/libmlic_$v.so; fi
  MLIC_HIP_LIB=$PWD/$L timeout -k 10 120 python -u tools/gpu/bench_dwpw.py 8 192 544 960 > "$OUT/b.tmp" 2>&1 || { echo "bench $v failed"; cat "$OUT/b.tmp"; exit 1; }
  echo "$v $(grep fused "$OUT/b.tmp")" | tee -a "$OUT/abl.log"
done
bash tools/gpu/pmc_dwpw.sh "$OUT/pmc" "8 192 544 960" dwpw2_kernel > "$OUT/pmc.log" 2>&1 || { echo "pmc failed"; tail -20 "$OUT/pmc.log"; exit 1; }
cat "$OUT/pmc.log"
