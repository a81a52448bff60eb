"""Latent-grid depthwise 3x3 (mlic_dw_run) against plain copies of the same bytes.
usage: python tools/gpu/dw_latent.py"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mlic_amd import _lib  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    dev = torch.device("cuda")
    st = torch.cuda.current_stream().cuda_stream
    P = C.c_void_p
    for (B, Cn, H, W) in ((8, 224, 68, 120), (8, 128, 68, 120), (8, 32, 68, 120), (8, 192, 136, 240), (16, 224, 32, 48)):
        x = torch.randn(B, Cn, H, W, device=dev)
        y = torch.empty_like(x)
        w = torch.randn(Cn, 9, device=dev) * 0.1
        b = torch.randn(Cn, device=dev) * 0.1
        f = lambda: _lib.call("mlic_dw_run", P(st), P(x.data_ptr()), P(w.data_ptr()), P(b.data_ptr()),  # noqa
                              P(y.data_ptr()), B, Cn, H, W, 1, 0)
        gb = 2 * x.numel() * 4 / 1e9
        res = {}
        for mode in (0, 1):
            _lib.call("mlic_set_kernel_option", b"dw_strip", mode)
            t = timeit(f)
            res[mode] = (t, y.clone())
        _lib.call("mlic_set_kernel_option", b"dw_strip", -1)
        same = torch.equal(res[0][1], res[1][1])
        tc = timeit(lambda: y.copy_(x))
        print(f"B={B} C={Cn} {H}x{W} ({gb * 1e3:.0f} MB r+w): tile {res[0][0] * 1e3:.1f} us {gb / res[0][0]:.0f} GB/s | "
              f"strip {res[1][0] * 1e3:.1f} us {gb / res[1][0]:.0f} GB/s (bit-equal {same}) | copy {tc * 1e3:.1f} us "
              f"{gb / tc:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
