"""Micro-benchmark of single conv layers through mlic_bench_conv (the model's kernel choice).

usage: python tools/gpu/bench_conv.py  [B Cin Cout H W K stride shuffle]...
Environment switches (MLIC_X4, MLIC_X4_RS, MLIC_X4_K, ...) select kernel variants.
"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mlic_amd import _lib  # noqa: E402

SHAPES = [  # the bench's heaviest conv layers (MLICPP_L, 1920x1088, 8 images per lane)
    (8, 192, 768, 272, 480, 3, 1, 1),  # g_s rbu subpel_conv / upsample (3rd stage)
    (8, 192, 768, 136, 240, 3, 1, 1),
    (8, 640, 6400, 68, 120, 1, 1, 0),  # hoisted EntropyParameters hyper columns
    (8, 320, 320, 68, 120, 5, 1, 0),   # global inter context reprojection
]


def main():
    shapes = SHAPES
    if len(sys.argv) > 1:
        v = [int(a) for a in sys.argv[1:]]
        shapes = [tuple(v[i:i + 8]) for i in range(0, len(v), 8)]
    ms, tf = C.c_double(), C.c_double()
    for B, ci, co, H, W, K, s, sh in shapes:
        _lib.call("mlic_bench_conv", 3, B, ci, co, H, W, K, s, sh, 10, C.byref(ms), C.byref(tf))
        print(f"B={B} {ci}->{co} {H}x{W} K={K} s={s} shuf={sh}: {ms.value:.3f} ms {tf.value:.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
