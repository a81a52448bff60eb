"""One conv shape through mlic_bench_conv (A/B timing and rocprofv3 PMC passes on the GPU box).

    python tools/conv_one.py impl B Cin Cout H W K stride shuffle [iters]

impl: 0 fp32 MFMA, 1 f16x3, 2 x3v2, 3 = what the model selects, 6 halo, 7 x4.
"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlic_amd import _lib  # noqa: E402


def main():
    a = [int(v) for v in sys.argv[1:]]
    impl, B, Cin, Cout, H, W, K, s, sh = a[:9]
    iters = a[9] if len(a) > 9 else 10
    ms, tf = C.c_double(), C.c_double()
    _lib.call("mlic_bench_conv", impl, B, Cin, Cout, H, W, K, s, sh, iters, C.byref(ms), C.byref(tf))
    print(f"impl{impl} B{B} {Cin}->{Cout} {H}x{W} k{K} s{s}: {ms.value:.3f} ms {tf.value:.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
