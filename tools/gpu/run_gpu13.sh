cd "$GRAFT_REPO_ROOT"
b() { timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 "$@"; }
b --lanes 4 > gpurun_out/b13_l4.json 2>>gpurun_out/b13.err || exit $?
b --lanes 8 > gpurun_out/b13_l8.json 2>>gpurun_out/b13.err || exit $?
MLIC_LANE_PRIORITY=0 b --lanes 4 > gpurun_out/b13_l4_noprio.json 2>>gpurun_out/b13.err || exit $?
b --lanes 4 --batch 16 > gpurun_out/b13_l4_b16.json 2>>gpurun_out/b13.err || exit $?
b --lanes 8 --batch 16 > gpurun_out/b13_l8_b16.json 2>>gpurun_out/b13.err || exit $?
echo done
