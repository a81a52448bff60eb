"""Per-kernel averages of the PMC counters in a rocprofv3 results DB (rocpd sqlite).

usage: python tools/pmc_summary.py <run_results.db> [kernel-substring]
Prints, per kernel name and counter, the mean value per dispatch and the dispatch count.
"""
import sqlite3
import sys
from collections import defaultdict


def summarize(db, filt=""):
    c = sqlite3.connect(db)
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for kname, cname, val, did in c.execute(
            "select kernel_name, counter_name, value, dispatch_id from counters_collection"):
        if filt and filt not in kname:
            continue
        acc[kname][cname] += val
        disp[kname].add(did)
    out = {}
    for k, cs in acc.items():
        n = len(disp[k])
        out[k] = {"dispatches": n, **{cn: v / n for cn, v in sorted(cs.items())}}
    return out


if __name__ == "__main__":
    res = summarize(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
    for k, d in res.items():
        print(k[:110])
        for cn, v in d.items():
            print(f"   {cn:32s} {v:,.0f}")
