"""Bitstream file format and the per-image evaluation harness.

File layout (utils/utils.py:28-83, utils/testing.py:203-262):
    >II   H, W of the unpadded image            (VBR: >III H, W, level)
    >III  h_z, w_z, n_strings (= 2)
    n_strings x ( >I length, bytes )            y stream, then z stream (image 0 only: B = 1)
Harness semantics (utils/testing.py:338-424) minus the NAIC "bpp > 0.1 => blur and retry" loop:
pad right/bottom with zeros to a multiple of 64, compress, write, read, decompress, crop;
bpp = 8 * filesize / (H * W) of the unpadded image; PSNR on uint8 images made by clamp(0,1)*255 and
truncation (torchvision ToPILImage), max 255 (utils/metrics.py:32-33).
"""
from __future__ import annotations

import io
import math
import struct
import time
from typing import Dict, List, Tuple

import torch
import torch.nn.functional as F


def file_bytes(y_len: int, z_len: int, vbr: bool = False) -> int:
    """Size of the file write_stream produces for one image's y and z streams (the header included:
    bpp_file = 8 * file_bytes / (H * W), utils/utils.py:71-83)."""
    return (12 if vbr else 8) + 12 + (4 + y_len) + (4 + z_len)


def write_stream(fd, H: int, W: int, shape, strings, level=None) -> int:
    n = 0
    if level is None:
        fd.write(struct.pack(">2I", H, W))
        n += 8
    else:
        fd.write(struct.pack(">3I", H, W, int(level)))
        n += 12
    fd.write(struct.pack(">3I", int(shape[0]), int(shape[1]), len(strings)))
    n += 12
    for s in strings:
        b = s[0]
        fd.write(struct.pack(">I", len(b)))
        fd.write(b)
        n += 4 + len(b)
    return n


def read_stream(fd, vbr: bool = False):
    hdr = struct.unpack(">3I" if vbr else ">2I", fd.read(12 if vbr else 8))
    hz, wz, n = struct.unpack(">3I", fd.read(12))
    strings: List[List[bytes]] = []
    for _ in range(n):
        (ln,) = struct.unpack(">I", fd.read(4))
        strings.append([fd.read(ln)])
    return hdr, strings, (hz, wz)


def write_file(path: str, H: int, W: int, out: Dict, level=None) -> int:
    with open(path, "wb") as f:
        return write_stream(f, H, W, out["shape"], out["strings"], level)


def read_file(path: str, vbr: bool = False):
    with open(path, "rb") as f:
        return read_stream(f, vbr)


def pad64(x: torch.Tensor) -> torch.Tensor:
    H, W = x.shape[-2:]
    ph = (64 - H % 64) % 64
    pw = (64 - W % 64) % 64
    return F.pad(x, (0, pw, 0, ph), mode="constant", value=0) if (ph or pw) else x


def to_u8(x: torch.Tensor) -> torch.Tensor:
    return (x.clamp(0, 1) * 255).to(torch.uint8)


def psnr_u8(a: torch.Tensor, b: torch.Tensor) -> float:
    mse = torch.mean((to_u8(a).float() - to_u8(b).float()) ** 2).item()
    return 20 * math.log10(255.0) - 10 * math.log10(mse) if mse > 0 else float("inf")


@torch.no_grad()
def code_image(net, img: torch.Tensor, **kw) -> Dict:
    """One image [1,3,H,W] in [0,1] through pad -> compress -> file bytes -> decompress -> crop."""
    assert img.dim() == 4 and img.size(0) == 1
    H, W = img.shape[-2:]
    x = pad64(img)
    t0 = time.time()
    out = net.compress(x, **kw)
    enc = time.time() - t0
    buf = io.BytesIO()
    level = kw.get("s") if kw else None
    nbytes = write_stream(buf, H, W, out["shape"], out["strings"], level)
    buf.seek(0)
    hdr, strings, shape = read_stream(buf, vbr=level is not None)
    t0 = time.time()
    dec = net.decompress(strings, shape, **kw)
    dect = time.time() - t0
    x_hat = dec["x_hat"][:, :, :H, :W]
    return {"H": H, "W": W, "bytes": nbytes, "bpp": 8.0 * nbytes / (H * W), "psnr": psnr_u8(img, x_hat),
            "enc_s": enc, "dec_s": dect, "x_hat": x_hat}
