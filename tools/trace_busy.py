"""GPU occupancy of a rocprofv3 kernel trace: the union of kernel [start, end] intervals against the
wall span, and the idle gaps by size.  usage: python tools/trace_busy.py run_kernel_trace.csv [t0_frac]"""
import csv
import sys


def main(path, skip=0.0):
    iv = []
    with open(path) as f:
        for r in csv.DictReader(f):
            iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    iv.sort()
    t0, t1 = iv[0][0], max(e for _, e, _ in iv)
    t0 = t0 + int(skip * (t1 - t0))
    busy, cur_s, cur_e, gaps = 0, None, None, []
    for s, e, _ in iv:
        if e <= t0:
            continue
        s = max(s, t0)
        if cur_e is None:
            cur_s, cur_e = s, e
        elif s > cur_e:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = t1 - t0
    print(f"span {span/1e6:.1f} ms  busy {busy/1e6:.1f} ms ({100*busy/span:.1f} %)  gaps {len(gaps)}")
    for lo, hi in ((0, 5e3), (5e3, 20e3), (20e3, 100e3), (100e3, 1e6), (1e6, 1e12)):
        sel = [g for g in gaps if lo <= g < hi]
        print(f"  gaps {lo/1e3:7.0f}-{hi/1e3:7.0f} us: {len(sel):6d}  {sum(sel)/1e6:8.2f} ms")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 0.0)
