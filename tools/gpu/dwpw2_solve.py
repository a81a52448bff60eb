"""dwpw2 bring-up failure, round 6 diagnosis: WHICH operand was wrong.

For the residual-only epilogue (epi = 64) the fused output is linear in the depthwise image:
y[:, p] = W t[:, p] + b + res[:, p].  A wrong pixel p gives d = y_fused - y_ref over all Cout channels,
and e = W^-1 d is the error of the pixel's depthwise operand if the MFMA's B operand was wrong (sparse e:
which channels, which k-step, hi or lo part), or a dense vector if the error entered after the products
(accumulator, residual, store).  Runs the given library (MLIC_HIP_LIB) on one shape up to `reps` times.

usage: python tools/gpu/dwpw2_solve.py B C H W [reps]"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mlic_amd import _lib  # noqa: E402


def main():
    B, Cn, H, W = [int(a) for a in sys.argv[1:5]]
    reps = int(sys.argv[5]) if len(sys.argv) > 5 else 4
    epi = 64
    g = torch.Generator().manual_seed(5)
    dev = torch.device("cuda")
    x = (torch.rand(B, Cn, H, W, generator=g) - 0.5).to(dev)
    dw = ((torch.rand(Cn, 1, 3, 3, generator=g) - 0.5) * 0.6).to(dev)
    db = (torch.rand(Cn, generator=g) - 0.5).to(dev)
    w = ((torch.rand(Cn, Cn, 1, 1, generator=g) - 0.5) * 0.2).to(dev)
    b = (torch.rand(Cn, generator=g) - 0.5).to(dev)
    res = (torch.rand(B, Cn, H, W, generator=g) - 0.5).to(dev)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = C.c_void_p
    _lib.call("mlic_set_kernel_option", b"dwpw2", 1)
    t = torch.full((B, Cn, H, W), float("nan"), device=dev)
    _lib.call("mlic_dw_run", st, P(x.data_ptr()), P(dw.data_ptr()), P(db.data_ptr()), P(t.data_ptr()), B, Cn, H, W, 1, 0)
    y2 = torch.full((B, Cn, H, W), float("nan"), device=dev)
    _lib.call("mlic_conv_run", st, 3, P(t.data_ptr()), P(w.data_ptr()), P(b.data_ptr()), P(y2.data_ptr()), B, Cn, Cn,
              H, W, 1, 1, epi, None, P(res.data_ptr()))
    torch.cuda.synchronize()
    W64 = w[:, :, 0, 0].double().cpu()
    Winv = torch.linalg.inv(W64)
    t_cpu = t.double().cpu()
    th = t.half().double().cpu()
    tl = (t - t.half().float()).half().double().cpu()
    for rep in range(reps):
        y = torch.full((B, Cn, H, W), float("nan"), device=dev)
        _lib.call("mlic_dwpw_run", st, P(x.data_ptr()), P(dw.data_ptr()), P(db.data_ptr()), P(w.data_ptr()),
                  P(b.data_ptr()), P(y.data_ptr()), B, Cn, Cn, H, W, epi, P(res.data_ptr()))
        torch.cuda.synchronize()
        bad = (y != y2)
        n = int(bad.sum())
        print(f"rep {rep}: {n} of {bad.numel()} differ", flush=True)
        if not n:
            continue
        pix = bad.any(dim=1).nonzero().tolist()  # (b, y, x)
        print(f"  {len(pix)} pixels; all Cout wrong at each: "
              f"{all(int(bad[bb, :, yy, xx].sum()) == Cn for bb, yy, xx in pix)}")
        for bb, yy, xx in pix[:6] + pix[-2:]:
            d = (y[bb, :, yy, xx] - y2[bb, :, yy, xx]).double().cpu()
            e = Winv @ d  # error of the pixel's depthwise operand, if that is where it entered
            big = (e.abs() > 1e-3 * max(1e-30, float(e.abs().max()))).nonzero().flatten().tolist()
            top = e.abs().argsort(descending=True)[:6].tolist()
            resid = float((W64 @ e - d).abs().max())
            tv = t_cpu[bb, :, yy, xx]
            print(f"  (b{bb} y{yy} x{xx}) |d| max {float(d.abs().max()):.3e}; e: {len(big)} channels above 1e-3 of max, "
                  f"top {[(c, round(float(e[c]), 6), round(float(tv[c]), 4), round(float(tl[bb, c, yy, xx]), 7)) for c in top]}")
            # is e = -(lo part) or -(hi part) of some channel block?  ratio e / t_lo and e / t_hi on the top channels
            rl = [round(float(e[c] / tl[bb, c, yy, xx]), 3) if float(tl[bb, c, yy, xx]) != 0 else None for c in top]
            rh = [round(float(e[c] / th[bb, c, yy, xx]), 3) for c in top]
            print(f"      e/t_lo {rl}  e/t_hi {rh}  (fit residual {resid:.2e})")
            # neighbour-pixel hypotheses: operand of another pixel in the same row
            cands = []
            for dx in (-16, 16, -32, 32):
                if 0 <= xx + dx < W:
                    cands.append((f"x{dx:+d}", float((th[bb, :, yy, xx + dx] + tl[bb, :, yy, xx + dx]
                                                      - th[bb, :, yy, xx] - tl[bb, :, yy, xx] - e).abs().max())))
            for dy in (-1, 1, -2, 2):
                if 0 <= yy + dy < H:
                    cands.append((f"y{dy:+d}", float((t_cpu[bb, :, yy + dy, xx] - t_cpu[bb, :, yy, xx] - e).abs().max())))
            print(f"      operand-from-neighbour fit (max |resid|): {cands}")
        break


if __name__ == "__main__":
    main()
