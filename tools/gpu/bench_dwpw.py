"""Micro-benchmark: fused depthwise+pointwise (mlic_dwpw_run) vs depthwise + resident pointwise.

usage: python tools/gpu/bench_dwpw.py [B C H W [epi]]   (default: the g_a stage-1 shape, 8 x 192 x 544 x 960,
epi 1 = GELU; 0 bias, 65 GELU + residual)
"""
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
    B, Cn, H, W = [int(a) for a in sys.argv[1:5]] if len(sys.argv) > 4 else (8, 192, 544, 960)
    epi = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(B, Cn, H, W, generator=g) - 0.5).to(dev)
    dw = (torch.rand(Cn, 9, generator=g) - 0.5).to(dev)
    db = (torch.rand(Cn, generator=g) - 0.5).to(dev)
    w = ((torch.rand(Cn, Cn, generator=g) - 0.5) * 0.2).to(dev)
    b = (torch.rand(Cn, generator=g) - 0.5).to(dev)
    y = torch.empty_like(x)
    res = torch.rand_like(x) if epi & 64 else None
    t = torch.empty_like(x)
    st = torch.cuda.current_stream().cuda_stream
    P = C.c_void_p
    fused = lambda: _lib.call("mlic_dwpw_run", P(st), P(x.data_ptr()), P(dw.data_ptr()), P(db.data_ptr()),  # noqa
                              P(w.data_ptr()), P(b.data_ptr()), P(y.data_ptr()), B, Cn, Cn, H, W, epi,
                              None if res is None else P(res.data_ptr()))
    dwk = lambda: _lib.call("mlic_dw_run", P(st), P(x.data_ptr()), P(dw.data_ptr()), P(db.data_ptr()),  # noqa
                            P(t.data_ptr()), B, Cn, H, W, 1, 0)
    pwk = lambda: _lib.call("mlic_conv_run", P(st), 3, P(t.data_ptr()), P(w.data_ptr()), P(b.data_ptr()),  # noqa
                            P(y.data_ptr()), B, Cn, Cn, H, W, 1, 1, 1, None, None)
    gb = 4.0 * B * Cn * H * W * 2 / 1e9
    tf, td, tp = timeit(fused), timeit(dwk), timeit(pwk)
    print(f"B={B} C={Cn} {H}x{W} epi={epi}: fused {tf:.3f} ms ({gb / tf:.0f} GB/s algorithmic)  dw {td:.3f} + pw {tp:.3f} = "
          f"{td + tp:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
