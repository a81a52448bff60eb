# linear attention: layer-table time with and without its contraction FLOPs (diagnostics build
# tools/gpu/libmlic_linabl.so, MLIC_LINATT_ABL=3)
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/linabl}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in base abl; do
  if [ $v = base ]; then L=mlic_amd/libmlic_hip.so; else L=tools/gpu/libmlic_linabl.so; fi
  MLIC_HIP_LIB=$PWD/$L timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --steps 1 --warmup 1 --layers-out "$OUT/layers_$v.tsv" > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err" || { echo "$v failed"; tail -20 "$OUT/bench_$v.err"; exit 1; }
  python3 - "$OUT/layers_$v.tsv" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1]), delimiter='\t'))
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    if r['kernel'] == 'linear_attention':
        k = 'inter' if 'inter' in r['layer'] else 'intra'
        agg[k][0] += int(r['launches']); agg[k][1] += float(r['ms'])
print(sys.argv[1], {k: (v[0], round(v[1], 3)) for k, v in agg.items()})
PY
done
