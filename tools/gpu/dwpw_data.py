"""Does the fused dwpw kernel's time depend on the data?  Same shape (8 x 192 x 544 x 960, GELU),
inputs / weights from different distributions.  usage: python tools/gpu/dwpw_data.py"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mlic_amd import _lib  # noqa: E402


def timeit(fn, iters=5):
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
    B, Cn, H, W = 8, 192, 544, 960
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    st = torch.cuda.current_stream().cuda_stream
    P = C.c_void_p
    y = torch.empty(B, Cn, H, W, device=dev)
    cases = {
        "uniform": lambda: torch.rand(B, Cn, H, W, generator=g, device=dev) - 0.5,
        "normal": lambda: torch.randn(B, Cn, H, W, generator=g, device=dev),
        "normal*10": lambda: torch.randn(B, Cn, H, W, generator=g, device=dev) * 10,
        "normal*0.01": lambda: torch.randn(B, Cn, H, W, generator=g, device=dev) * 0.01,
        "zeros": lambda: torch.zeros(B, Cn, H, W, device=dev),
        "ones": lambda: torch.ones(B, Cn, H, W, device=dev),
        "smooth": lambda: torch.sin(torch.arange(H * W, device=dev, dtype=torch.float32) * 0.001).reshape(1, 1, H, W)
        .expand(B, Cn, H, W).contiguous(),
    }
    for wname, ws in (("w0.1", 0.1), ("w0.01", 0.01)):
        dw = ((torch.rand(Cn, 9, generator=g, device=dev) - 0.5) * 2 * ws)
        db = (torch.rand(Cn, generator=g, device=dev) - 0.5) * ws
        w = ((torch.rand(Cn, Cn, generator=g, device=dev) - 0.5) * 2 * ws)
        b = (torch.rand(Cn, generator=g, device=dev) - 0.5) * ws
        for name, mk in cases.items():
            x = mk()
            for mode in (1, 0):
                f = lambda: _lib.call("mlic_dwpw_run", P(st), P(x.data_ptr()), P(dw.data_ptr()), P(db.data_ptr()),  # noqa
                                      P(w.data_ptr()), P(b.data_ptr()), P(y.data_ptr()), B, Cn, Cn, H, W, mode, None)
                print(f"{wname} {name:12s} mode {mode}: {timeit(f):.3f} ms", flush=True)
            del x


if __name__ == "__main__":
    main()
