"""LocalContext module at a given latent size: packed-attention + x4 fusion path (precision 2) vs the
unfolded path (precision 1), same weights and input."""
import sys
import torch
sys.path.insert(0, ".")
from mlic_amd import get_model, synthetic

H, W = int(sys.argv[1]), int(sys.argv[2])
B = int(sys.argv[3]) if len(sys.argv) > 3 else 1
net = get_model("MLICPP_L")
net.load_state_dict(synthetic.synth_state_dict("MLICPP_L", 0))
net = net.cuda().eval()
g = torch.Generator().manual_seed(0)
x = (torch.randn(B, 32, H, W, generator=g) * 3).cuda()
outs = []
for prec in (2, 1):
    net.set_precision(prec)
    y = net.run_module("local", 0, x, None, out_shape=(B, 64, H, W))
    torch.cuda.synchronize()
    outs.append(y)
d = (outs[0] - outs[1]).abs()
print(H, W, B, "max", d.max().item(), "scale", outs[1].abs().max().item())
idx = torch.nonzero(d > 1e-3 * outs[1].abs().max())
print("bad", idx.shape[0], idx[:10].tolist())
