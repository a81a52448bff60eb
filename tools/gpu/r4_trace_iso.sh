# per-dispatch kernel trace of one isolated step (one lane, 8 images), compacted; plus split A/B
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/triso; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o run -- \
  python3 -u bench.py --lanes 1 --batch 8 --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $OUT/bench.json 2> $OUT/bench.err || { echo fail $?; tail $OUT/bench.err; exit 1; }
f=$(ls $OUT/tr/*kernel_trace.csv $OUT/tr/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 - "$f" $OUT/iso_dispatches.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
with open(sys.argv[2], "w") as o:
    o.write("start_ns,dur_ns,grid,wg,lds,vgpr,agpr,scratch,name\n")
    for r in rows:
        g = f'{r.get("Grid_Size_X","")}x{r.get("Grid_Size_Y","")}x{r.get("Grid_Size_Z","")}'
        w = r.get("Workgroup_Size_X", "")
        o.write(f'{r["Start_Timestamp"]},{int(r["End_Timestamp"]) - int(r["Start_Timestamp"])},{g},{w},{r.get("LDS_Block_Size", r.get("Lds_Size",""))},{r.get("VGPR_Count","")},{r.get("Accum_VGPR_Count","")},{r.get("Scratch_Size","")},"{r["Kernel_Name"][:160]}"\n')
print(len(rows), "dispatches;", list(rows[0].keys()))
PY
rm -rf $OUT/tr; gzip -f $OUT/iso_dispatches.csv
run() { tag=$1; shift; timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag failed $?"; tail -5 $OUT/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/$tag.json').readline()); print('$tag', d['value'], d['ms_per_step'], d['host_thread_ms_per_step'])"; }
run s4l2 --split 4 --lanes 2 && run s2l4 --split 2 --lanes 4 && run s8l2 --split 8 --lanes 2 --group-concurrency 8 && run s4l3 --split 4 --lanes 3 && run s4l4 --split 4 --lanes 4 && run s4l2b --split 4 --lanes 2
