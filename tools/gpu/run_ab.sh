cd "$GRAFT_REPO_ROOT"
b() { timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/ab_$1.json 2>/dev/null || exit 1; python -c "import json; d=json.load(open('gpurun_out/ab_$1.json')); print('$1', d['value'], d['ms_per_step'], d['kernel_families_ms_isolated_share'].get('local_attn_kernel'))"; }
b packed1
MLIC_LA_PACKED=0 b unpacked
b packed2
MLIC_LA_PACKED=0 b unpacked2
