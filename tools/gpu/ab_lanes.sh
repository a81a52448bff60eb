# lane count A/B of the default workload (no profiled passes); usage: bash tools/gpu/ab_lanes.sh
cd "$GRAFT_REPO_ROOT"
for l in ${LANES:-2 4 6 8}; do
  timeout -k 10 300 python3 -u bench.py --lanes $l --steps 3 --warmup 1 --no-roofline --no-cpu-baseline 2>/dev/null \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('lanes', $l, d['value'], d['ms_per_step'], d['wall_ms_per_step'])" \
    || { echo "lanes $l failed"; exit 1; }
done
