# Alternating A/B of environment arms on one bench configuration (timed steps only, no profiled
# passes): the default and each arm, REPS times, in one process sequence on one box -- the only
# comparison the box-to-box spread allows.  usage on the box:
#   CONFIG=main ARGS="--split 4 --lanes 2" REPS=2 bash tools/gpu/ab_env.sh "MLIC_X4_SPLITK=1" "MLIC_HOIST=1"
# An arm is a space-free list of VAR=VAL assignments joined by ',' (e.g. "MLIC_POOL_PRIO=0,MLIC_LANES=3").
cd "$GRAFT_REPO_ROOT"; OUT=${OUT:-gpurun_out/ab_env}; mkdir -p "$OUT"
run() {
  local tag=$1
  env ${tag//,/ } timeout -k 10 300 python3 -u bench.py --config "${CONFIG:-main}" --steps ${STEPS:-5} --warmup 2 \
    --no-cpu-baseline --no-roofline $ARGS > "$OUT/b.json" 2> "$OUT/b.err" || { echo "$tag failed"; tail -5 "$OUT/b.err"; return 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b.json').readline()); print('${CONFIG:-main}', '$tag', d['value'], d['ms_per_step'])"
}
for rep in $(seq ${REPS:-2}); do
  run MLIC_DEFAULT=1 || exit 1
  for a in "$@"; do run "$a" || exit 1; done
done
