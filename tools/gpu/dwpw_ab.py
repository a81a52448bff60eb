"""Fused dwpw launch time per epilogue mode at the g_a / g_s full-resolution shape (8 x 192 x 544 x 960),
for A/B between library builds (MLIC_HIP_LIB).  usage: python tools/gpu/dwpw_ab.py [tag]"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mlic_amd import _lib  # noqa: E402


def timeit(fn, iters=10):
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
    tag = sys.argv[1] if len(sys.argv) > 1 else ""
    B, Cn, H, W = 8, 192, 544, 960
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(B, Cn, H, W, generator=g) - 0.5).to(dev)
    r = (torch.rand(B, Cn, H, W, generator=g) - 0.5).to(dev)
    dw = (torch.rand(Cn, 9, generator=g) - 0.5).to(dev)
    db = (torch.rand(Cn, generator=g) - 0.5).to(dev)
    w = ((torch.rand(Cn, Cn, generator=g) - 0.5) * 0.2).to(dev)
    b = (torch.rand(Cn, generator=g) - 0.5).to(dev)
    y = torch.empty_like(x)
    st = torch.cuda.current_stream().cuda_stream
    P = C.c_void_p
    outs = {}
    epis = [int(e) for e in os.environ.get("DWPW_EPI", "0,1,65").split(",")]  # (one mode for PMC passes)
    for epi in epis:
        res = P(r.data_ptr()) if epi & 64 else None
        f = lambda: _lib.call("mlic_dwpw_run", P(st), P(x.data_ptr()), P(dw.data_ptr()), P(db.data_ptr()),  # noqa
                              P(w.data_ptr()), P(b.data_ptr()), P(y.data_ptr()), B, Cn, Cn, H, W, epi, res)
        t = timeit(f)
        outs[epi] = float(y.double().sum().item())
        print(f"{tag} epi={epi}: {t:.3f} ms  checksum {outs[epi]:.6e}", flush=True)


if __name__ == "__main__":
    main()
