import sys, torch
sys.path.insert(0, '.'); sys.path.insert(0, 'oracle')
import numpy as np
import mlic_ref_cpu as ref
from mlic_amd import get_model, synthetic
dev = torch.device("cuda:0")
g = np.load("tests/golden/modules_L.npz")
sd = synthetic.synth_state_dict("MLICPP_L", 0)
net = get_model("MLICPP_L"); net.load_state_dict(sd); net = net.to(dev).eval()
m = ref.RefMLIC("MLICPP_L", sd)
x = torch.from_numpy(g["lrpn2_in"])
res = torch.randn(1, 32, 8, 12, generator=torch.Generator().manual_seed(5))
exp = res + ref.ckbd_nonanchor(m.lrp(x, "nonanchor", 2))
for trial in range(3):
    got = net.run_module("lrpn", 2, x.to(dev), res.to(dev), out_shape=(1, 32, 8, 12)).cpu()
    d = (got - exp).abs()
    print("trial", trial, "maxdiff", float(d.max()), "anchor-pos maxdiff", float(ref.ckbd_anchor(d).max()),
          "got-res at nonanchor", float(ref.ckbd_nonanchor(got - res).abs().max()))
# with zero residual
got0 = net.run_module("lrpn", 2, x.to(dev), torch.zeros(1, 32, 8, 12, device=dev), out_shape=(1, 32, 8, 12)).cpu()
e0 = ref.ckbd_nonanchor(m.lrp(x, "nonanchor", 2))
print("zero-res maxdiff", float((got0 - e0).abs().max()))
print(got0[0, 0, :3, :6]); print(e0[0, 0, :3, :6])
