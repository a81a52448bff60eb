# bisect a parity failure over the round's x4 switches: direct 1x1 B rows, the 224-row tile
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/bisect}
T=${2:-test_vbr_4k_mixed}
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in "MLIC_X4_DIRECT=1" "MLIC_X4_DIRECT=0" "MLIC_X4_BM224=0" "MLIC_X4_BM96=0" "MLIC_X4_DIRECT=0 MLIC_X4_BM224=0 MLIC_X4_BM96=0"; do
  n=$(echo $cfg | tr ' =' '__')
  env $cfg timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 380 --timeout-method thread -k "$T" > "$OUT/$n.log" 2>&1
  rc=$?
  echo "$cfg rc=$rc $(tail -1 $OUT/$n.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
