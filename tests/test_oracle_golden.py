"""Pin the CPU oracle (oracle/mlic_ref_cpu.py) against fixtures produced by running
the reference itself (oracle/gen_golden.py).  CPU only."""
import hashlib
import math

import numpy as np
import pytest
import torch

import mlic_ref_cpu as ref
from mlic_amd import spec, synthetic


def sd_sha(sd):
    h = hashlib.sha256()
    for k in sorted(sd):
        h.update(k.encode())
        h.update(sd[k].contiguous().numpy().tobytes())
    return h.hexdigest()


def close(a, b, rtol=1e-5, atol=1e-5):
    a = torch.as_tensor(np.asarray(a)).float()
    b = torch.as_tensor(np.asarray(b)).float()
    assert a.shape == b.shape, (a.shape, b.shape)
    err = (a - b).abs().max().item()
    lim = (atol + rtol * b.abs()).min().item()
    assert torch.allclose(a, b, rtol=rtol, atol=atol), f"max abs err {err}"


def test_ckbd_bitexact(golden):
    g = golden("ckbd.npz")
    y = torch.from_numpy(g["y"])
    assert torch.equal(ref.ckbd_anchor(y), torch.from_numpy(g["anchor"]))
    assert torch.equal(ref.ckbd_nonanchor(y), torch.from_numpy(g["nonanchor"]))
    assert torch.equal(ref.ckbd_squeeze(y, True), torch.from_numpy(g["sq_anchor"]))
    assert torch.equal(ref.ckbd_squeeze(y, False), torch.from_numpy(g["sq_nonanchor"]))
    assert torch.equal(ref.ckbd_unsqueeze(y[..., :4], True), torch.from_numpy(g["unsq_anchor"]))
    assert torch.equal(ref.ckbd_unsqueeze(y[..., :4], False), torch.from_numpy(g["unsq_nonanchor"]))


def test_local_mask_bitexact(golden):
    g = golden("masks.npz")
    for k in g.files:
        if k.startswith("mask_"):
            H, W = map(int, k[5:].split("x"))
            assert torch.equal(ref.local_attn_mask(H, W), torch.from_numpy(g[k])), k
    assert np.array_equal(synthetic.relative_position_index(5), g["relative_position_index"])


def test_scale_table_and_indexes_bitexact(golden):
    g = golden("scale_table.npz")
    t = ref.scale_table()
    assert torch.equal(t, torch.from_numpy(g["table"]))
    idx = ref.build_indexes(torch.from_numpy(g["sweep"]), t)
    assert torch.equal(idx, torch.from_numpy(g["sweep_indexes"]))


def test_module_vectors(golden):
    g = golden("modules_L.npz")
    sd = synthetic.synth_state_dict("MLICPP_L", 0)
    assert sd_sha(sd) == str(g["sd_sha"])
    m = ref.RefMLIC("MLICPP_L", sd)
    T = lambda k: torch.from_numpy(g[k])
    with torch.no_grad():
        close(m.local_context(T("lc_in"), 0), g["lc_out"])
        close(m.channel_context(T("chan3_in"), 3), g["chan3_out"])
        close(m.inter_context(T("chan3_in"), 3), g["inter3_out"])
        close(m.inter_context(T("inter9_in"), 9), g["inter9_out"], rtol=1e-4, atol=1e-4)
        close(m.intra_context(T("intra_in1"), T("intra_in2"), 1), g["intra_out"])
        close(m.entropy_parameters(T("epa2_in"), "anchor", 2), g["epa2_out"])
        close(m.lrp(T("lrpn2_in"), "nonanchor", 2), g["lrpn2_out"])
        close(m.rbu(T("rbu1_in"), "g_s.synthesis_transform.1"), g["rbu1_out"], rtol=1e-4, atol=1e-4)
        close(m.rbws(T("rbws0_in"), "g_a.analysis_transform.0", True), g["rbws0_out"])
        lik = ref.gaussian_likelihood(T("gc_y"), T("gc_s"), T("gc_m"))
        assert torch.equal(lik, T("gc_lik"))
        close(m.eb_likelihood(T("eb_in")), g["eb_lik"], rtol=1e-5, atol=1e-7)


FWD = [("MLICPP_L", 128, 192, None), ("MLICPP_L", 128, 128, None), ("MLICPP_S", 128, 128, None),
       ("MLICPP_S2", 128, 128, None), ("MLICPP_M", 128, 128, None), ("MLICPP_M_SMALL_DEC", 128, 128, None),
       ("MLICPP_L_VBR", 128, 128, 0), ("MLICPP_L_VBR", 128, 128, 3), ("MLICPP_L_VBR", 128, 128, 5),
       ("MLICPP_S_VBR", 128, 128, 0), ("MLICPP_S_VBR", 128, 128, 3), ("MLICPP_S_VBR", 128, 128, 5),
       ("MLICPP_M_SMALL_DEC_VBR", 128, 128, 0), ("MLICPP_M_SMALL_DEC_VBR", 128, 128, 3)]


@pytest.mark.parametrize("name,H,W,s", FWD)
def test_forward_matches_reference(golden, name, H, W, s):
    tag = f"{name}_{H}x{W}" + ("" if s is None else f"_s{s}")
    g = golden(f"forward_{tag}.npz")
    sd = synthetic.synth_state_dict(name, 0)
    assert sd_sha(sd) == str(g["sd_sha"]), "synthetic weights drifted from the fixture"
    img_seed = 1 if (name == "MLICPP_L" and W == 128) else 0
    x = synthetic.synth_image(H, W, img_seed)
    assert hashlib.sha256(x.numpy().tobytes()).hexdigest() == str(g["x_sha"])
    m = ref.RefMLIC(name, sd)
    out = m.forward(x, s=1 if s is None else s)
    yl, zl = out["likelihoods"]["y_likelihoods"], out["likelihoods"]["z_likelihoods"]
    bpp = ref.bpp_from_likelihoods(yl, zl, H * W)
    assert abs(bpp - float(g["bpp"])) < 1e-4
    close(out["x_hat"], g["x_hat"], rtol=1e-4, atol=1e-4)
    close(zl, g["z_lik"], rtol=1e-4, atol=1e-7)
    close(yl, g["y_lik"], rtol=1e-3, atol=1e-6)
    psnr_ref = ref.psnr_uint8(x, torch.from_numpy(g["x_hat"]))
    assert abs(ref.psnr_uint8(x, out["x_hat"]) - psnr_ref) < 0.01


@pytest.mark.parametrize("name,H,W,s,img", [("MLICPP_L", 128, 192, None, 0), ("MLICPP_S", 128, 128, None, 0),
                                            ("MLICPP_M_SMALL_DEC", 128, 128, None, 0), ("MLICPP_S_VBR", 128, 128, 0, 0),
                                            ("MLICPP_S_VBR", 128, 128, 3, 0), ("MLICPP_S_VBR", 128, 128, 5, 0),
                                            ("MLICPP_S_VBR", 192, 256, 1, 3), ("MLICPP_M_SMALL_DEC_VBR", 128, 128, 0, 0),
                                            ("MLICPP_M_SMALL_DEC_VBR", 128, 128, 3, 0)])
def test_compress_streams_match_reference(golden, name, H, W, s, img):
    """Coder inputs (y symbols / indexes, z symbols) vs the reference's.  VBR: the fixture holds the
    values a consistent codec codes, taken from the reference forward itself (oracle/gen_golden.py
    vbr_streams; the reference's own VBR compress is defective)."""
    g = golden(f"forward_{name}_{H}x{W}" + ("" if s is None else f"_s{s}") + ".npz")
    sd = synthetic.synth_state_dict(name, 0)
    m = ref.RefMLIC(name, sd)
    x = synthetic.synth_image(H, W, img)
    assert hashlib.sha256(x.numpy().tobytes()).hexdigest() == str(g["x_sha"])
    kw = {} if s is None else {"s": s}
    st = m.compress_streams(x, **kw)
    sym = torch.cat([p[0].reshape(-1) for p in st["phases"]]).numpy()
    idx = torch.cat([p[1].reshape(-1) for p in st["phases"]]).numpy()
    assert np.array_equal(st["z_symbols"].numpy(), g["z_symbols"])
    assert np.array_equal(idx, g["y_indexes"])
    assert np.array_equal(sym, g["y_symbols"])
    # decode from the streams reproduces the forward x_hat (round trip invariant)
    dec = m.decode_streams(st["z_symbols"], [p[0] for p in st["phases"]], **kw)
    assert torch.equal(dec["y_hat"], st["y_hat"])
    close(dec["x_hat"], g["x_hat"], rtol=1e-4, atol=1e-4)


# realistic-rate weight sets (synthetic.RATE_LAMBDAS stand-ins, 0.06-0.9 bpp): forward and the exact
# coder inputs, oracle vs the reference (oracle/gen_golden.py "rates")
RATES = [("MLICPP_L", 0, None), ("MLICPP_L", 2, None), ("MLICPP_L", 5, None), ("MLICPP_S", 1, None),
         ("MLICPP_M_SMALL_DEC", 1, None), ("MLICPP_L_VBR", 2, 1), ("MLICPP_M_SMALL_DEC_VBR", 1, 2)]


@pytest.mark.parametrize("name,rate,s", RATES)
def test_rate_sets_match_reference(golden, name, rate, s):
    H, W = 192, 256
    tag = f"{name}_{H}x{W}" + ("" if s is None else f"_s{s}") + f"_r{rate}"
    g = golden(f"forward_{tag}.npz")
    sd = synthetic.synth_state_dict(name, rate=rate)
    assert sd_sha(sd) == str(g["sd_sha"]), "synthetic weights drifted from the fixture"
    x = synthetic.synth_image(H, W, 3)
    assert hashlib.sha256(x.numpy().tobytes()).hexdigest() == str(g["x_sha"])
    m = ref.RefMLIC(name, sd)
    out = m.forward(x, s=1 if s is None else s)
    yl, zl = out["likelihoods"]["y_likelihoods"], out["likelihoods"]["z_likelihoods"]
    assert abs(ref.bpp_from_likelihoods(yl, zl, H * W) - float(g["bpp"])) < 1e-4
    close(out["x_hat"], g["x_hat"], rtol=1e-4, atol=1e-4)
    if "y_symbols" in g.files:
        st = m.compress_streams(x, **({} if s is None else {"s": s}))
        sym = torch.cat([p[0].reshape(-1) for p in st["phases"]]).numpy()
        idx = torch.cat([p[1].reshape(-1) for p in st["phases"]]).numpy()
        assert np.array_equal(st["z_symbols"].numpy(), g["z_symbols"])
        assert np.array_equal(idx, g["y_indexes"])
        assert np.array_equal(sym, g["y_symbols"])


def test_reference_batch_stream_order(golden):
    """The reference codes a B > 1 batch into ONE y stream (mlicpp.py:215, 279-281): its coder inputs are
    each image's phase streams interleaved phase-major, image-minor (the order mlic_batch_stream codes).
    Checked against the reference's own list for a 3-image batch (oracle/gen_golden.py gen_batch_streams)."""
    g = golden("batch_streams_MLICPP_S_3x128x192.npz")
    assert int(g["n_y_strings"]) == 1 and int(g["n_z_strings"]) == 3
    name = "MLICPP_S"
    m = ref.RefMLIC(name, synthetic.synth_state_dict(name, 0))
    per = [m.compress_streams(synthetic.synth_image(128, 192, int(s_))) for s_ in g["seeds"]]
    sym = np.concatenate([per[b]["phases"][k][0].reshape(-1).numpy()
                          for k in range(len(per[0]["phases"])) for b in range(len(per))])
    idx = np.concatenate([per[b]["phases"][k][1].reshape(-1).numpy()
                          for k in range(len(per[0]["phases"])) for b in range(len(per))])
    assert np.array_equal(idx, g["y_indexes"])
    assert np.array_equal(sym, g["y_symbols"])
