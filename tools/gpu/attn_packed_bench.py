"""Packed LocalContext attention micro-benchmark (mlic_local_attn_packed_run) at the MLICPP_L latent
size, 8 images: ms per launch by HIP events.  usage: python tools/gpu/attn_packed_bench.py [B]"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mlic_amd import _lib, synthetic  # noqa: E402


def main():
    B, H, W = int(sys.argv[1]) if len(sys.argv) > 1 else 8, 68, 120
    dev = torch.device("cuda")
    qkv = torch.randn(B, 96, H, W, device=dev)
    table = torch.randn(81, 2, device=dev)
    index = torch.from_numpy(synthetic.relative_position_index(5)).reshape(-1).to(torch.int32).to(dev)
    npos = (H * W + 31) // 32 * 32
    out = torch.empty(B, 25, npos, 64, dtype=torch.int16, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    args = (C.c_void_p(st), C.c_void_p(qkv.data_ptr()), C.c_void_p(table.data_ptr()), C.c_void_p(index.data_ptr()),
            C.c_void_p(out.data_ptr()), H, W, B, 0.25)
    _lib.call("mlic_local_attn_packed_run", *args)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    a.record()
    for _ in range(n):
        _lib.call("mlic_local_attn_packed_run", *args)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / n
    gb = (4.0 * B * H * W * 96 + 2.0 * B * 25 * npos * 64) / 1e9
    print(f"packed attention B={B}: {ms * 1e3:.1f} us/launch  {gb / ms * 1e3:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
