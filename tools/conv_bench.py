"""Conv kernel micro-benchmark over the MLICPP_L layer shapes that dominate the step (GPU box)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlic_amd import _lib  # noqa: E402

# (name, B, Cin, Cout, H, W, K, stride, shuffle) — 1080p, per-GPU batch 8
SHAPES = [
    ("g_s.5 subpel 3x3 192->768 @272x480", 8, 192, 768, 272, 480, 3, 1, 1),
    ("g_s.3 subpel 3x3 192->768 @136x240", 8, 192, 768, 136, 240, 3, 1, 1),
    ("g_s/g_a pw 192->192 @544x960", 8, 192, 192, 544, 960, 1, 1, 0),
    ("pw 192->192 @272x480", 8, 192, 192, 272, 480, 1, 1, 0),
    ("EP 960->320 @68x120", 8, 960, 320, 68, 120, 1, 1, 0),
    ("EP 320->256 @68x120", 8, 320, 256, 68, 120, 1, 1, 0),
    ("inter9 reproj 5x5 288->96 @68x120", 8, 288, 96, 68, 120, 5, 1, 0),
    ("LRP pw 608->224 @68x120", 8, 608, 224, 68, 120, 1, 1, 0),
]


EXTRA = [("g_s.7 subpel 3x3 192->12 @544x960", 8, 192, 12, 544, 960, 3, 1, 1),
         ("g_a.0 skip 1x1/2 3->192 @1088x1920", 8, 3, 192, 1088, 1920, 1, 2, 0),
         ("g_a.0 pw 3->192 @544x960", 8, 3, 192, 544, 960, 1, 1, 0)]


def main():
    impls = [int(a) for a in sys.argv[1:]] or [0, 1]
    for name, B, Cin, Cout, H, W, K, s, sh in SHAPES + EXTRA:
        row = [f"{name:40s}"]
        for impl in impls:
            if impl == 6 and not (K in (1, 3, 5) and s == 1 and Cout >= 32 and Cin >= 32):
                row.append(f"impl{impl}: {'-':>8s}")
                continue
            ms, tf = C.c_double(), C.c_double()
            _lib.call("mlic_bench_conv", impl, B, Cin, Cout, H, W, K, s, sh, 10, C.byref(ms), C.byref(tf))
            Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
            gbs = 4.0 * B * (Cin * H * W + Cout * Ho * Wo) / (ms.value * 1e-3) / 1e9
            row.append(f"impl{impl}: {ms.value:8.3f} ms {tf.value:7.1f} TF/s {gbs:6.0f} GB/s")
        print("  ".join(row), flush=True)


if __name__ == "__main__":
    main()
