# hardware queues / per-phase D2H placement A/B on the main and Kodak configs (timed steps only)
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/hwq; mkdir -p $OUT
run() { cfg=$1; shift; tag="$*"; env "$@" timeout -k 10 300 python3 -u bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > $OUT/b.json 2> $OUT/b.err || { echo "$cfg $tag fail"; tail -5 $OUT/b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b.json').readline()); print('$cfg $tag', d['value'], d['ms_per_step'])"; }
for rep in 1 2; do
  run main GPU_MAX_HW_QUEUES=4 MLIC_PHASE_D2H=1 && run main GPU_MAX_HW_QUEUES=16 MLIC_PHASE_D2H=1 && run main GPU_MAX_HW_QUEUES=4 MLIC_PHASE_D2H=0 && run main GPU_MAX_HW_QUEUES=16 MLIC_PHASE_D2H=0 || exit 1
done
for rep in 1 2; do
  run kodak GPU_MAX_HW_QUEUES=4 MLIC_PHASE_D2H=1 && run kodak GPU_MAX_HW_QUEUES=16 MLIC_PHASE_D2H=1 && run kodak GPU_MAX_HW_QUEUES=4 MLIC_PHASE_D2H=0 && run kodak GPU_MAX_HW_QUEUES=4 MLIC_DW_STRIP=0 || exit 1
done
