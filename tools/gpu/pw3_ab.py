"""Full-resolution GDN / IGDN 1x1 launch time (8 x 192 x 544 x 960, + residual): pw_resident (pw3 off) vs the
register-row kernel's pointwise form (pw3 on), alternating.  usage: python tools/gpu/pw3_ab.py"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mlic_amd import _lib  # noqa: E402

GDN, IGDN, RES, SQUARE = 2, 4, 64, 256


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
    B, Cn, H, W = [int(v) for v in os.environ.get("PW3_SHAPE", "8,192,544,960").split(",")]
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(0)
    x = ((torch.rand(B, Cn, H, W, generator=g) - 0.5) * 4).to(dev)
    r = (torch.rand(B, Cn, H, W, generator=g) - 0.5).to(dev)
    w = ((torch.rand(Cn, Cn, 1, 1, generator=g) - 0.5).abs() * 0.01).to(dev)
    b = (1.0 + torch.rand(Cn, generator=g)).to(dev)
    y = torch.empty_like(x)
    st = torch.cuda.current_stream().cuda_stream
    P = C.c_void_p
    for rnd in range(2):
        for on in (0, 1):
            _lib.call("mlic_set_kernel_option", b"pw3", on)
            for epi in [int(e, 0) for e in os.environ.get("PW3_EPI", "0x142,0x144").split(",")]:
                f = lambda: _lib.call("mlic_conv_run", P(st), 3, P(x.data_ptr()), P(w.data_ptr()), P(b.data_ptr()),  # noqa
                                      P(y.data_ptr()), B, Cn, Cn, H, W, 1, 1, epi, P(x.data_ptr()), P(r.data_ptr()))
                t = timeit(f)
                print(f"pw3={on} epi={epi:#x}: {t:.3f} ms  checksum {float(y.double().sum().item()):.6e}", flush=True)
    _lib.call("mlic_set_kernel_option", b"pw3", -1)


if __name__ == "__main__":
    main()
