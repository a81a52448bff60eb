"""Packed LocalContext attention output digest (seeded inputs, several grids), to compare two builds'
bits: python tools/gpu/la_hash.py [save-prefix]  (MLIC_HIP_LIB selects the library)."""
import ctypes as C
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mlic_amd import _lib, synthetic  # noqa: E402


def main():
    dev = torch.device("cuda")
    h = hashlib.sha256()
    for B, H, W in [(8, 68, 120), (2, 24, 40), (1, 13, 21), (3, 34, 60)]:
        g = torch.Generator().manual_seed(B * 1000 + H)
        qkv = (torch.randn(B, 96, H, W, generator=g) * 2).to(dev)
        table = torch.randn(81, 2, generator=g).to(dev)
        index = torch.from_numpy(synthetic.relative_position_index(5)).reshape(-1).to(torch.int32).to(dev)
        npos = (H * W + 31) // 32 * 32
        out = torch.zeros(B, 25, npos, 64, dtype=torch.int16, device=dev)
        st = torch.cuda.current_stream().cuda_stream
        _lib.call("mlic_local_attn_packed_run", C.c_void_p(st), C.c_void_p(qkv.data_ptr()),
                  C.c_void_p(table.data_ptr()), C.c_void_p(index.data_ptr()), C.c_void_p(out.data_ptr()),
                  H, W, B, 0.25)
        torch.cuda.synchronize()
        h.update(out.cpu().numpy().tobytes())
        if len(sys.argv) > 1 and B < 8:
            import numpy as np
            np.save(f"{sys.argv[1]}_{B}x{H}x{W}.npy", out.cpu().numpy())
    print("la_hash", h.hexdigest(), flush=True)


if __name__ == "__main__":
    main()
