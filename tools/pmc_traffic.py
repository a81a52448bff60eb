"""HBM traffic per launch of one kernel from rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE are
collected in separate passes, MI355X_MICROARCH.md §rocprofv3 PMC slots).

    python tools/pmc_traffic.py <fetch_dir> <write_dir> <kernel-substring> <out.json> [key=value ...]

FETCH_SIZE / WRITE_SIZE are in KiB (TCC_EA0 requests).  gfx950 caveat (MI355X_MICROARCH.md §HBM):
FETCH_SIZE reads exactly half the bytes of a 16-byte-per-lane streaming read; other access widths
are uncalibrated, so we report the raw sum and, separately, the sum with FETCH doubled (upper bound).
Infinity-Cache hits are counted too (they are memory-side requests).
"""
import csv
import glob
import json
import os
import sys


def per_launch(d, counter, kernel):
    vals = []
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            if r["Counter_Name"] == counter and kernel.replace(" ", "") in r["Kernel_Name"].replace(" ", ""):
                vals.append(float(r["Counter_Value"]) * 1024.0)
    return sum(vals) / len(vals) if vals else None, len(vals)


def main():
    fetch_dir, write_dir, kernel, out = sys.argv[1:5]
    extra = dict(kv.split("=", 1) for kv in sys.argv[5:])
    for k in ("H", "W", "batch"):
        if k in extra:
            extra[k] = int(extra[k])
    f, nf = per_launch(fetch_dir, "FETCH_SIZE", kernel)
    w, nw = per_launch(write_dir, "WRITE_SIZE", kernel)
    res = dict(extra, kernel=kernel, launches_fetch=nf, launches_write=nw,
               fetch_bytes_per_launch=f, write_bytes_per_launch=w,
               # MI355X_MICROARCH.md §HBM: FETCH_SIZE counts half the bytes of 16-B/lane streaming reads
               # (this kernel's operand loads are 16-B/lane) -> doubled; WRITE_SIZE is exact
               conv_hbm_bytes_per_launch=(2 * f + w) if f is not None and w is not None else None,
               conv_hbm_bytes_per_launch_raw=(f + w) if f is not None and w is not None else None)
    # the keys bench.py's --traffic-json reads (roofline.traffic of the dominant family)
    res["family"] = kernel
    res["hbm_bytes_per_launch"] = res["conv_hbm_bytes_per_launch"]
    res["method"] = ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of bench.py --steps 1 "
                     "--warmup 0 --no-roofline; mean over every launch of the family; FETCH doubled "
                     "(MI355X_MICROARCH.md HBM: gfx950 tallies 128-B reads at 64 B), WRITE as is; "
                     "Infinity-Cache hits included")
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
