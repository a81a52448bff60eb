# round 6: staggered stream priorities across the concurrent request streams' models (default) vs equal (MLIC_GROUP_PRIO=0)
cd "$GRAFT_REPO_ROOT"; OUT=${OUT:-gpurun_out/r6gp}; mkdir -p $OUT
timeout -k 10 60 python3 -c "
import ctypes as C, torch
h=C.CDLL('libamdhip64.so'); lo=C.c_int(); hi=C.c_int(); print('priority range rc', h.hipDeviceGetStreamPriorityRange(C.byref(lo), C.byref(hi)), 'least', lo.value, 'greatest', hi.value)" || exit 1
OUT=$OUT ARGS="--no-decode-record" REPS=3 STEPS=4 bash tools/gpu/ab_env.sh "MLIC_GROUP_PRIO=0" || exit 1
echo "schedule streams:"
OUT=$OUT ARGS="--no-decode-record --schedule streams" REPS=2 STEPS=4 bash tools/gpu/ab_env.sh "MLIC_GROUP_PRIO=0"
