"""Generate tests/golden/*.npz by running the REFERENCE itself (read-only
/root/reference/MLIC++, through oracle/refshim) on CPU.

Run in the dev container only:  python -B oracle/gen_golden.py
The fixtures are data (inputs + expected outputs); the reference source never
leaves this container.  Weights come from mlic_amd.synthetic.synth_state_dict
(seeded, conditioned), images from mlic_amd.synthetic.synth_image; each fixture
records a checksum of both so a drift in the generators is caught by the tests.
"""
from __future__ import annotations

import hashlib
import math
import os
import sys

sys.dont_write_bytecode = True
_HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(_HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, _HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import refload  # noqa: E402
from mlic_amd import spec, synthetic  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
torch.cuda.synchronize = lambda *a, **k: None   # reference compress() calls it unconditionally
torch.set_num_threads(8)


def sd_checksum(sd):
    h = hashlib.sha256()
    for k in sorted(sd):
        h.update(k.encode())
        h.update(sd[k].detach().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()


def t_checksum(t):
    return hashlib.sha256(t.detach().cpu().contiguous().numpy().tobytes()).hexdigest()


def save(name, **arrs):
    path = os.path.join(OUT, name)
    np.savez_compressed(path, **{k: (v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v))
                                 for k, v in arrs.items()})
    print("wrote", path, os.path.getsize(path), "bytes")


def gen_bitexact():
    ck = refload.load_module("utils/ckbd.py")
    g = torch.Generator().manual_seed(7)
    y = torch.randn(2, 3, 6, 8, generator=g)
    save("ckbd.npz", y=y, anchor=ck.ckbd_anchor(y), nonanchor=ck.ckbd_nonanchor(y),
         sq_anchor=ck.ckbd_anchor_sequeeze(y), sq_nonanchor=ck.ckbd_nonanchor_sequeeze(y),
         unsq_anchor=ck.ckbd_anchor_unsequeeze(y[..., :4]), unsq_nonanchor=ck.ckbd_nonanchor_unsequeeze(y[..., :4]))
    ctx = refload.load_module("modules/transform/context.py")
    masks = {}
    for (H, W) in ((8, 8), (6, 10), (4, 6), (8, 12)):
        lc = ctx.LocalContext(dim=32)
        lc.update_resolution(H, W, "cpu")
        masks[f"mask_{H}x{W}"] = lc.attn_mask
    masks["relative_position_index"] = ctx.LocalContext(dim=32).relative_position_index
    save("masks.npz", **masks)
    func = refload.load_module("utils/func.py")
    table = func.get_scale_table()
    ent = sys.modules["compressai.entropy_models"]
    gc = ent.GaussianConditional(None)
    gc.update_scale_table(table)
    sweep = torch.cat([table, table * (1 + 1e-7), table * (1 - 1e-7), torch.tensor([0.0, -1.0, 0.05, 0.11, 1e3]),
                       torch.exp(torch.linspace(-3, 6, 257))])
    save("scale_table.npz", table=table, quantized_cdf=gc.quantized_cdf, offset=gc.offset,
         cdf_length=gc.cdf_length, sweep=sweep, sweep_indexes=gc.build_indexes(sweep))


def _ref_model(name, seed, rate=None):
    m = refload.build(name)
    sd = synthetic.synth_state_dict(name, seed, rate=rate)
    m.load_state_dict(sd)
    return m.eval(), sd


def gen_modules():
    """Module-level vectors for MLICPP_L seed 0 on an 8x12 latent."""
    name = "MLICPP_L"
    m, sd = _ref_model(name, 0)
    g = torch.Generator().manual_seed(11)
    H, W = 8, 12
    C = 32
    arr = {"sd_sha": sd_checksum(sd)}
    with torch.no_grad():
        xa = torch.randn(1, C, H, W, generator=g) * 3
        ck = refload.load_module("utils/ckbd.py")
        xa_anchor = ck.ckbd_anchor(xa)
        arr["lc_in"] = xa_anchor
        arr["lc_out"] = m.local_context[0](xa_anchor)
        prev = torch.randn(1, C * 3, H, W, generator=g) * 3
        arr["chan3_in"] = prev
        arr["chan3_out"] = m.channel_context[3](prev)
        arr["inter3_out"] = m.global_inter_context[3](prev)
        prev9 = torch.randn(1, C * 9, H, W, generator=g) * 3
        arr["inter9_in"] = prev9
        arr["inter9_out"] = m.global_inter_context[9](prev9)
        x1 = torch.randn(1, C, H, W, generator=g) * 3
        arr["intra_in1"] = x1
        arr["intra_in2"] = xa_anchor
        arr["intra_out"] = m.global_intra_context[1](x1, xa_anchor)
        ep_in = torch.randn(1, 832, H, W, generator=g)
        arr["epa2_in"] = ep_in
        arr["epa2_out"] = m.entropy_parameters_anchor[2](ep_in)
        lrp_in = torch.randn(1, 320 + 3 * C, H, W, generator=g)
        arr["lrpn2_in"] = lrp_in
        arr["lrpn2_out"] = m.lrp_nonanchor[2](lrp_in)
        rbu_in = torch.randn(1, 320, H, W, generator=g)
        arr["rbu1_in"] = rbu_in
        arr["rbu1_out"] = m.g_s.synthesis_transform[1](rbu_in)
        rbws_in = torch.rand(1, 3, 2 * H, 2 * W, generator=g)
        arr["rbws0_in"] = rbws_in
        arr["rbws0_out"] = m.g_a.analysis_transform[0](rbws_in)
        gc_y = torch.randn(1, C, H, W, generator=g) * 4
        gc_s = torch.randn(1, C, H, W, generator=g) * 2
        gc_m = torch.randn(1, C, H, W, generator=g)
        arr["gc_y"], arr["gc_s"], arr["gc_m"] = gc_y, gc_s, gc_m
        arr["gc_out"], arr["gc_lik"] = m.gaussian_conditional(gc_y, gc_s, gc_m)
        z = torch.randn(2, 192, 2, 3, generator=g) * 3
        arr["eb_in"] = z
        arr["eb_out"], arr["eb_lik"] = m.entropy_bottleneck(z)
    save("modules_L.npz", **arr)
    m.update(force=True)
    save("eb_cdf_L.npz", quantized_cdf=m.entropy_bottleneck.quantized_cdf,
         offset=m.entropy_bottleneck.offset, cdf_length=m.entropy_bottleneck.cdf_length,
         sd_sha=sd_checksum(sd))


EB_SETS = [("MLICPP_L", None)] + [("MLICPP_L", r) for r in range(6)] + [
    ("MLICPP_S", None), ("MLICPP_S", 1), ("MLICPP_S2", None), ("MLICPP_M", None), ("MLICPP_M_SMALL_DEC", None),
    ("MLICPP_M_SMALL_DEC", 1), ("MLICPP_S_VBR", None), ("MLICPP_L_VBR", 2)]


def gen_eb():
    """EntropyBottleneck.update() tables (the z coder's CDFs) of every fixture weight set."""
    arr = {}
    for name, rate in EB_SETS:
        m, sd = _ref_model(name, 0, rate)
        m.update(force=True)
        eb = m.entropy_bottleneck
        tag = name + ("" if rate is None else f"_r{rate}")
        arr[f"{tag}.quantized_cdf"] = eb.quantized_cdf
        arr[f"{tag}.offset"] = eb.offset
        arr[f"{tag}.cdf_length"] = eb.cdf_length
        arr[f"{tag}.sd_sha"] = sd_checksum(sd)
    save("eb_cdf_sets.npz", **arr)


def _vbr_capture(m):
    """Record, during one reference VBR forward (mlicpp_vbr.py:245-330, stage 2, no_quantoffset), the
    input of every ste_round and the scaled scales handed to gaussian_conditional."""
    mod = sys.modules[type(m).__module__]
    rounds, gc_scales = [], []
    orig = mod.ste_round

    def rec_round(t):
        rounds.append(t.detach().clone())
        return orig(t)
    mod.ste_round = rec_round
    hook = m.gaussian_conditional.register_forward_hook(lambda mo, inp, out: gc_scales.append(inp[1].detach().clone()))
    return rounds, gc_scales, lambda: (setattr(mod, "ste_round", orig), hook.remove())


def vbr_streams(m, rounds, gc_scales):
    """The coder inputs of a consistent VBR codec, from the reference forward's own values: phase
    (slice i, anchor) codes round((y - mu) * scale) at the anchor cells in ckbd squeeze order
    (utils/ckbd.py:47-73), with index build_indexes(scale * sigma) -- the indexes the reference's
    compress_anchor_vbr computes (ckbd.py:81); its symbols (ckbd.py:87, which subtracts mu twice and
    never scales) are the documented defect this replaces.  rounds[0] is the z rounding."""
    ck = refload.load_module("utils/ckbd.py")
    sym, idx = [], []
    S = len(gc_scales)
    assert len(rounds) == 1 + 2 * S, (len(rounds), S)
    for i in range(S):
        for ph, sq in ((0, ck.ckbd_anchor_sequeeze), (1, ck.ckbd_nonanchor_sequeeze)):
            sym.append(torch.round(sq(rounds[1 + 2 * i + ph])).int().reshape(-1))
            idx.append(m.gaussian_conditional.build_indexes(sq(gc_scales[i])).reshape(-1))
    z_sym = torch.round(rounds[0]).int()
    return torch.cat(sym).numpy(), torch.cat(idx).numpy().astype(np.int32), z_sym


def gen_forward(name, H, W, seed=0, img_seed=0, s=None, with_streams=False, rate=None):
    m, sd = _ref_model(name, seed, rate)
    x = synthetic.synth_image(H, W, img_seed)
    vbr_rec = None
    if s is not None and with_streams:
        vbr_rec = _vbr_capture(m)
    with torch.no_grad():
        out = m(x) if s is None else m(x, stage=2, s=s)
    yl, zl = out["likelihoods"]["y_likelihoods"], out["likelihoods"]["z_likelihoods"]
    bpp = float(sum(torch.log(l).sum() / (-math.log(2) * H * W) for l in (yl, zl)))
    arr = dict(x_hat=out["x_hat"], y_lik=yl, z_lik=zl, bpp=bpp, sd_sha=sd_checksum(sd), x_sha=t_checksum(x))
    if vbr_rec is not None:
        rounds, gc_scales, undo = vbr_rec
        undo()
        m.update(force=True)
        arr["y_symbols"], arr["y_indexes"], arr["z_symbols"] = vbr_streams(m, rounds, gc_scales)
        arr["z_shape"] = np.asarray([H // 64, W // 64], np.int32)
    elif with_streams:
        m.update(force=True)
        enc_mod = sys.modules[type(m).__module__]
        captured = {}

        class Enc:
            def encode_with_indexes(self, symbols, indexes, cdf, lengths, offsets):
                captured["sym"], captured["idx"] = symbols, indexes

            def flush(self):
                return b""
        enc_mod.BufferedRansEncoder = Enc
        with torch.no_grad():
            c = m.compress(x)
        arr["y_symbols"] = np.asarray(captured["sym"], np.int32)
        arr["y_indexes"] = np.asarray(captured["idx"], np.int32)
        arr["z_symbols"] = torch.stack([s_[1] for s_ in c["strings"][1]])
        arr["z_shape"] = np.asarray(list(c["shape"]), np.int32)
    tag = f"{name}_{H}x{W}" + ("" if s is None else f"_s{s}") + ("" if rate is None else f"_r{rate}")
    save(f"forward_{tag}.npz", **arr)
    print(f"  {tag}: bpp={bpp:.4f}")


def gen_batch_streams(name="MLICPP_S", H=128, W=192, seeds=(40, 41, 42)):
    """The reference's coder inputs for a B > 1 batch (mlicpp.py:215, 279-281): ONE symbol / index
    list for the whole batch, in its own order (phase-major, image-minor), and the z symbols."""
    m, sd = _ref_model(name, 0)
    m.update(force=True)
    x = torch.cat([synthetic.synth_image(H, W, s_) for s_ in seeds])
    enc_mod = sys.modules[type(m).__module__]
    captured = {}

    class Enc:
        def encode_with_indexes(self, symbols, indexes, cdf, lengths, offsets):
            captured["sym"], captured["idx"] = symbols, indexes

        def flush(self):
            return b""
    enc_mod.BufferedRansEncoder = Enc
    with torch.no_grad():
        c = m.compress(x)
    save(f"batch_streams_{name}_{len(seeds)}x{H}x{W}.npz", y_symbols=np.asarray(captured["sym"], np.int32),
         y_indexes=np.asarray(captured["idx"], np.int32), n_y_strings=len(c["strings"][0]),
         n_z_strings=len(c["strings"][1]), seeds=np.asarray(seeds), sd_sha=sd_checksum(sd), x_sha=t_checksum(x))


def main():
    os.makedirs(OUT, exist_ok=True)
    what = sys.argv[1:] or ["bitexact", "modules", "forward", "rates", "eb", "svbr", "sdvbr", "batch"]
    if "eb" in what:
        gen_eb()
    if "svbr" in what:
        # MLICPP_S_VBR, the VBR name the reference factory registers (models/model_loader.py:12-13)
        for s in (0, 3, 5):
            gen_forward("MLICPP_S_VBR", 128, 128, s=s, with_streams=True)
        gen_forward("MLICPP_S_VBR", 192, 256, img_seed=3, s=1, with_streams=True)
    if "batch" in what:
        gen_batch_streams()
    if "sdvbr" in what:
        # MLICPP_M_SMALL_DEC_VBR (models/model_loader.py:14-15, models/mlicpp_sd_vbr.py)
        for s in (0, 3):
            gen_forward("MLICPP_M_SMALL_DEC_VBR", 128, 128, s=s, with_streams=True)
        gen_forward("MLICPP_M_SMALL_DEC_VBR", 192, 256, img_seed=3, rate=1, s=2, with_streams=True)
    if "bitexact" in what:
        gen_bitexact()
    if "modules" in what:
        gen_modules()
    if "forward" in what:
        gen_forward("MLICPP_L", 128, 192, with_streams=True)
        gen_forward("MLICPP_L", 128, 128, img_seed=1)
        gen_forward("MLICPP_S", 128, 128, with_streams=True)
        gen_forward("MLICPP_S2", 128, 128)
        gen_forward("MLICPP_M", 128, 128)
        gen_forward("MLICPP_M_SMALL_DEC", 128, 128, with_streams=True)
        for s in (0, 3, 5):
            gen_forward("MLICPP_L_VBR", 128, 128, s=s)
    if "rates" in what:
        # realistic-rate weight sets (synthetic.RATE_LAMBDAS stand-ins): 0.1-0.7 bpp, coder streams
        for r in (0, 2, 5):
            gen_forward("MLICPP_L", 192, 256, img_seed=3, rate=r, with_streams=True)
        gen_forward("MLICPP_S", 192, 256, img_seed=3, rate=1, with_streams=True)
        gen_forward("MLICPP_M_SMALL_DEC", 192, 256, img_seed=3, rate=1, with_streams=True)
        gen_forward("MLICPP_L_VBR", 192, 256, img_seed=3, rate=2, s=1)


if __name__ == "__main__":
    main()
