# dwpw k-loop unrolled (default build) vs rolled (-DMLIC_DWPW_ROLLED) + the dwpw GPU tests
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/dwu; mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 120 python3 -u tools/gpu/dwpw_ab.py unrolled 2>&1 | grep -v amdgpu.ids || exit 1
  MLIC_HIP_LIB=$PWD/mlic_amd/libmlic_hip_rolled.so timeout -k 10 120 python3 -u tools/gpu/dwpw_ab.py rolled 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 120 --timeout-method thread -k "dwpw" 2>&1 | tail -3
# Kodak-size regression hunt: the register-strip depthwise and the coder-pool order
OUT=gpurun_out/kod; mkdir -p $OUT
for v in "MLIC_POOL_PRIO=2" "MLIC_POOL_PRIO=0" "MLIC_POOL_PRIO=2" "MLIC_POOL_PRIO=0"; do
  env $v timeout -k 10 300 python3 -u bench.py --config kodak --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > $OUT/k.json 2> $OUT/k.err || { echo kodak fail; tail -5 $OUT/k.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/k.json').readline()); print('kodak $v', d['value'], d['ms_per_step'], d['wall_ms_per_step'])"
done
