# the parity-suite sequence that ran before a VBR 4K round-trip mismatch, default switches then the
# packed 1x1 path
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/vbrseq}
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in "MLIC_X4_DIRECT=1" "MLIC_X4_DIRECT=0"; do
  n=$(echo $cfg | tr ' =' '__')
  env $cfg timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -k "vbr or 4k or config_size or bpp_lik" > "$OUT/$n.log" 2>&1
  rc=$?
  echo "$cfg rc=$rc $(tail -1 $OUT/$n.log)"
  grep -E "AssertionError|^E .*\(" "$OUT/$n.log" | head -5
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
