"""Where the packed LocalContext attention differs from the MFMA kernel (debug)."""
import ctypes as C
import sys
import torch
sys.path.insert(0, ".")
from mlic_amd import _lib, synthetic
H, W, B = 68, 120, 1
g = torch.Generator().manual_seed(5)
dev = torch.device("cuda")
ch = 32
qkv = (torch.randn(B, 3 * ch, H, W, generator=g) * 2).to(dev)
table = torch.randn(81, 2, generator=g).to(dev)
index = torch.from_numpy(synthetic.relative_position_index(5)).reshape(-1).to(torch.int32).to(dev)
scale = 16 ** -0.5
st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
ref = torch.full((B, 25 * ch, H, W), float("nan"), device=dev)
_lib.call("mlic_local_attn_run", st, 1, C.c_void_p(qkv.data_ptr()), C.c_void_p(table.data_ptr()),
          C.c_void_p(index.data_ptr()), C.c_void_p(ref.data_ptr()), ch, H, W, B, float(scale))
npos = (H * W + 31) // 32 * 32
out = torch.zeros(B, 25, npos, 64, dtype=torch.float16, device=dev)
_lib.call("mlic_local_attn_packed_run", st, C.c_void_p(qkv.data_ptr()), C.c_void_p(table.data_ptr()),
          C.c_void_p(index.data_ptr()), C.c_void_p(out.data_ptr()), H, W, B, float(scale))
v = out[..., :32].float() + out[..., 32:].float()
v = v[:, :, :H * W].permute(0, 3, 1, 2).reshape(B, 25 * ch, H, W)
d = (v - ref).abs()
print("max", d.max().item(), "mean", d.mean().item())
bad = torch.nonzero(d > 1e-5 * ref.abs().max())
print("bad count", bad.shape[0])
for b_, r, y, x in bad[:20].tolist():
    print(" row", r, "(c", r // 25, "cell", r % 25, ") pix", y, x, "ref", ref[b_, r, y, x].item(), "got", v[b_, r, y, x].item())
