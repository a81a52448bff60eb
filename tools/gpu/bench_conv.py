"""Micro-benchmark of single conv layers through mlic_bench_conv.

usage: python tools/gpu/bench_conv.py [--latent] [B Cin Cout H W K stride epi]...
epi = Epi flags (common.h: 1 GELU, 8 tanh/2, 16/32 mask, 64 residual, 128 shuffle).
$MLIC_BENCH_IMPL forces a kernel family (CONV_* id: 2 x3v2, 3 pw_resident, 7 x4); default the
model's choice.  Environment switches (MLIC_X4, MLIC_X4_RS, MLIC_X4_K, ...) select variants.
"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mlic_amd import _lib  # noqa: E402

SHAPES = [  # the bench's heaviest conv layers (MLICPP_L, 1920x1088, 8 images per lane)
    (8, 192, 768, 272, 480, 3, 1, 128),  # g_s rbu subpel_conv / upsample (3rd stage)
    (8, 192, 768, 136, 240, 3, 1, 128),
    (8, 640, 6400, 68, 120, 1, 1, 0),  # hoisted EntropyParameters hyper columns
    (8, 320, 320, 68, 120, 5, 1, 0),   # global inter context reprojection
]

LATENT = [  # latent-resolution 1x1 convs (MLICPP_L, 1920x1088 -> 68x120, 8 images)
    (8, 224, 128, 68, 120, 1, 1, 1),    # LRP .2
    (8, 128, 32, 68, 120, 1, 1, 8 | 16 | 64),  # LRP head: tanh/2, mask, residual
    (8, 96, 192, 68, 120, 1, 1, 1),     # channel context .0 (i = 3)
    (8, 192, 128, 68, 120, 1, 1, 1),    # channel context .2
    (8, 128, 128, 68, 120, 1, 1, 0),    # channel context .4
    (8, 96, 96, 68, 120, 1, 1, 0),      # inter q/k/v (i = 3)
    (8, 32, 32, 68, 120, 1, 1, 0),      # intra q/k/v
    (8, 32, 96, 68, 120, 1, 1, 0),      # local qkv_proj
    (8, 64, 64, 68, 120, 1, 1, 0),      # local proj
    (8, 96, 128, 68, 120, 1, 1, 1),     # inter mlp.0
    (8, 128, 64, 68, 120, 1, 1, 64),    # mlp.4 + residual
    (8, 96, 64, 68, 120, 1, 1, 0),      # inter skip
]


def main():
    args = sys.argv[1:]
    shapes = SHAPES
    if args and args[0] == "--latent":
        shapes, args = LATENT, args[1:]
    if args:
        v = [int(a) for a in args]
        shapes = [tuple(v[i:i + 8]) for i in range(0, len(v), 8)]
    impl = int(os.environ.get("MLIC_BENCH_IMPL", "-1"))
    ms, tf = C.c_double(), C.c_double()
    for B, ci, co, H, W, K, s, epi in shapes:
        _lib.call("mlic_bench_conv", impl, B, ci, co, H, W, K, s, epi, 10, C.byref(ms), C.byref(tf))
        gbs = 4.0 * B * H * W * (ci + co * (2 if epi & 64 else 1)) / (ms.value * 1e-3) / 1e9
        print(f"impl={impl} B={B} {ci}->{co} {H}x{W} K={K} s={s} epi={epi}: {ms.value * 1e3:.1f} us "
              f"{tf.value:.1f} TF/s {gbs:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
