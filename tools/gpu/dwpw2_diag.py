"""Mismatch locations of the fused dwpw launch against depthwise + resident pointwise (bring-up aid).
usage: python tools/gpu/dwpw2_diag.py B C H W epi"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mlic_amd import _lib  # noqa: E402


def main():
    B, Cn, H, W, epi = [int(a) for a in sys.argv[1:6]]
    g = torch.Generator().manual_seed(5)
    dev = torch.device("cuda")
    x = (torch.rand(B, Cn, H, W, generator=g) - 0.5).to(dev)
    dw = ((torch.rand(Cn, 1, 3, 3, generator=g) - 0.5) * 0.6).to(dev)
    db = (torch.rand(Cn, generator=g) - 0.5).to(dev)
    w = ((torch.rand(Cn, Cn, 1, 1, generator=g) - 0.5) * 0.2).to(dev)
    b = (torch.rand(Cn, generator=g) - 0.5).to(dev)
    res = (torch.rand(B, Cn, H, W, generator=g) - 0.5).to(dev)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.call("mlic_set_kernel_option", b"dwpw2", int(os.environ.get("MLIC_DWPW2", "1")))
    P = C.c_void_p
    y = torch.full((B, Cn, H, W), float("nan"), device=dev)
    _lib.call("mlic_dwpw_run", st, P(x.data_ptr()), P(dw.data_ptr()), P(db.data_ptr()), P(w.data_ptr()),
              P(b.data_ptr()), P(y.data_ptr()), B, Cn, Cn, H, W, epi, P(res.data_ptr()))
    t = torch.full((B, Cn, H, W), float("nan"), device=dev)
    _lib.call("mlic_dw_run", st, P(x.data_ptr()), P(dw.data_ptr()), P(db.data_ptr()), P(t.data_ptr()), B, Cn, H, W, 1, 0)
    y2 = torch.full((B, Cn, H, W), float("nan"), device=dev)
    repi = epi & ~64 if os.environ.get("D2_REF_NORES") == "1" else epi  # a build that skips the residual
    _lib.call("mlic_conv_run", st, 3, P(t.data_ptr()), P(w.data_ptr()), P(b.data_ptr()), P(y2.data_ptr()), B, Cn, Cn,
              H, W, 1, 1, repi, None, P(res.data_ptr()))
    torch.cuda.synchronize()
    bad = (y != y2) & ~(torch.isnan(y) & torch.isnan(y2))
    n = int(bad.sum())
    print(f"MLIC_DWPW2={os.environ.get('MLIC_DWPW2')} B={B} C={Cn} {H}x{W} epi={epi}: {n} of {bad.numel()} differ; nan in fused {int(torch.isnan(y).sum())}")
    if n:
        idx = bad.nonzero()
        for k, name in enumerate("bcyx"):
            vals, cnt = idx[:, k].unique(return_counts=True)
            print(f"  {name}: {len(vals)} distinct, first {vals[:12].tolist()} counts {cnt[:12].tolist()}")
        d = (y - y2).abs()[bad]
        print(f"  |diff| max {float(d.max()):.3e} mean {float(d.mean()):.3e}")


if __name__ == "__main__":
    main()
