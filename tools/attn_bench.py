"""LocalContext attention micro-benchmark (GPU box): both kernels at the MLICPP_L latent size."""
import ctypes as C
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlic_amd import _lib, synthetic  # noqa: E402


def main():
    B, ch, H, W = int(sys.argv[1]) if len(sys.argv) > 1 else 16, 32, 68, 120
    dev = torch.device("cuda")
    qkv = torch.randn(B, 3 * ch, H, W, device=dev)
    table = torch.randn(81, 2, device=dev)
    index = torch.from_numpy(synthetic.relative_position_index(5)).reshape(-1).to(torch.int32).to(dev)
    out = torch.empty(B, 25 * ch, H, W, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    for impl in (0, 1):
        args = (C.c_void_p(st), impl, C.c_void_p(qkv.data_ptr()), C.c_void_p(table.data_ptr()),
                C.c_void_p(index.data_ptr()), C.c_void_p(out.data_ptr()), ch, H, W, B, 0.25)
        _lib.call("mlic_local_attn_run", *args)
        t0 = time.perf_counter()
        n = 20
        for _ in range(n):
            _lib.call("mlic_local_attn_run", *args)
        ms = (time.perf_counter() - t0) / n * 1e3
        fl = B * H * W * 2 * 2 * 25 * 25 * (ch // 2) * 2
        gb = 4.0 * B * H * W * (3 * ch + 25 * ch) / 1e9
        print(f"impl{impl}: {ms:.3f} ms/call (incl. sync)  {fl / ms / 1e9:.1f} TF/s  {gb / ms * 1e3:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
