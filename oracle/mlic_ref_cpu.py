"""ORACLE — test infrastructure only.  CPU fp32 restatement of the MLIC++ hot path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / CPU baseline.  The product (mlic_amd) never
imports it; the HIP path fails loudly when its extension is missing.

It is a functional restatement over a plain state_dict (no nn.Module tree) of:

  forward ............ MLIC++/models/mlicpp.py:79-185 (+ SD: mlicpp_small_decoder.py:86-192,
                       VBR stage 2: mlicpp_vbr.py:137-519 with no_quantoffset=True)
  compress symbols ... mlicpp.py:199-290 + utils/ckbd.py:123-144 (the symbol/index
                       streams handed to the rANS coder, in coder order)
  decode ............. mlicpp.py:292-378 + ckbd.py:195-220, fed by a symbol source
  layers ............. modules/layers/{conv,res_blk,attention}.py,
                       modules/transform/{analysis,synthesis,context,entropy,quantization}.py
  compressai 1.2.6 ... GDN, GaussianConditional (likelihood / build_indexes), EntropyBottleneck
                       likelihood, quantize_ste — restated from the published library; compressai
                       is not in this image, so these are pinned only through the reference's call
                       sites and the fixtures in tests/golden (see DESIGN.md "parity").

It follows the reference's floating-point operation order so that the fixtures
produced by running the reference itself (oracle/gen_golden.py) are matched to
~1e-6.  Pinned by tests/test_oracle_golden.py.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

from mlic_amd import spec

T = torch.Tensor


# ----------------------------------------------------------------------------- ckbd
def ckbd_anchor(y: T) -> T:
    """utils/ckbd.py:35-39 — anchor = (h + w) odd."""
    out = torch.zeros_like(y)
    out[:, :, 0::2, 1::2] = y[:, :, 0::2, 1::2]
    out[:, :, 1::2, 0::2] = y[:, :, 1::2, 0::2]
    return out


def ckbd_nonanchor(y: T) -> T:
    """utils/ckbd.py:41-45 — non-anchor = (h + w) even."""
    out = torch.zeros_like(y)
    out[:, :, 0::2, 0::2] = y[:, :, 0::2, 0::2]
    out[:, :, 1::2, 1::2] = y[:, :, 1::2, 1::2]
    return out


def ckbd_squeeze(y: T, anchor: bool) -> T:
    """ckbd.py:47-59: [B,C,H,W] -> [B,C,H,W/2] keeping anchor (or non-anchor) cells."""
    B, C, H, W = y.shape
    out = torch.zeros(B, C, H, W // 2, dtype=y.dtype)
    a, b = (1, 0) if anchor else (0, 1)
    out[:, :, 0::2, :] = y[:, :, 0::2, a::2]
    out[:, :, 1::2, :] = y[:, :, 1::2, b::2]
    return out


def ckbd_unsqueeze(s: T, anchor: bool) -> T:
    """ckbd.py:61-73: inverse of ckbd_squeeze, zero elsewhere."""
    B, C, H, W2 = s.shape
    out = torch.zeros(B, C, H, W2 * 2, dtype=s.dtype)
    a, b = (1, 0) if anchor else (0, 1)
    out[:, :, 0::2, a::2] = s[:, :, 0::2, :]
    out[:, :, 1::2, b::2] = s[:, :, 1::2, :]
    return out


# ----------------------------------------------------------------------------- masks / tables
def local_attn_mask(H: int, W: int, window: int = 5) -> T:
    """context.py:43-65: mask[p, i, j] = 0 if window cells i and j of position p are both
    in-bounds anchor cells, else -100 (built with a zero-padded unfold of the ckbd map)."""
    ck = torch.zeros(1, 1, H, W)
    ck[:, :, 0::2, 1::2] = 1
    ck[:, :, 1::2, 0::2] = 1
    win = F.unfold(ck, kernel_size=window, padding=(window - 1) // 2)[0].t()  # [L, 25]
    m = win[:, :, None] * win[:, None, :]
    return m.masked_fill(m == 0.0, -100.0).masked_fill(m == 1.0, 0.0)


def scale_table() -> T:
    """utils/func.py:16-19."""
    return torch.exp(torch.linspace(math.log(0.11), math.log(256), 64))


def build_indexes(scales: T, table: T, bound: float = 0.11) -> T:
    """compressai GaussianConditional.build_indexes: 63 - #{t in table[:-1] : s' <= t}."""
    s = torch.max(scales, torch.tensor([bound], dtype=torch.float32))
    idx = torch.full(s.shape, len(table) - 1, dtype=torch.int32)
    for t in table[:-1]:
        idx -= (s <= t).int()
    return idx


def std_cumulative(x: T) -> T:
    return 0.5 * torch.erfc(float(-(2 ** -0.5)) * x)


def gaussian_likelihood(inputs: T, scales: T, means: T) -> T:
    """compressai GaussianConditional.forward in eval mode (dequantize + _likelihood + bound)."""
    outputs = torch.round(inputs - means) + means
    values = torch.abs(outputs - means)
    s = torch.max(scales, torch.tensor([0.11], dtype=torch.float32))
    lik = std_cumulative((0.5 - values) / s) - std_cumulative((-0.5 - values) / s)
    return torch.max(lik, torch.tensor([1e-9], dtype=torch.float32))


# ----------------------------------------------------------------------------- the model
class RefMLIC:
    """Stateless-weights restatement of MLICPlusPlus / MLICPlusPlusSD / MLICPlusPlusVbr."""

    def __init__(self, name: str, state_dict: Dict[str, T]):
        self.cfg = spec.get_config(name)
        self.sd = {k: v.detach().to("cpu") for k, v in state_dict.items()}
        self._mask_cache = {}

    # -- primitives -----------------------------------------------------------
    def w(self, k):
        return self.sd[k]

    def conv(self, x, p, stride=1, padding=None, groups=1):
        wt = self.sd[f"{p}.weight"]
        if padding is None:
            padding = wt.shape[-1] // 2
        return F.conv2d(x, wt, self.sd.get(f"{p}.bias"), stride=stride, padding=padding, groups=groups)

    def dwsep(self, x, p, stride=1):
        x = self.conv(x, f"{p}.depth_conv", stride=stride, groups=x.shape[1])
        return self.conv(x, f"{p}.point_conv")

    def conv3x3(self, x, p, stride=1, dw=True):
        return self.dwsep(x, p, stride) if dw else self.conv(x, p, stride=stride)

    def gdn(self, x, p, inverse):
        def reparam(v, name):
            b = self.sd[f"{p}.{name}_reparam.lower_bound.bound"]
            ped = self.sd[f"{p}.{name}_reparam.pedestal"]
            return torch.max(v, b) ** 2 - ped
        C = x.shape[1]
        beta = reparam(self.sd[f"{p}.beta"], "beta")
        gamma = reparam(self.sd[f"{p}.gamma"], "gamma").reshape(C, C, 1, 1)
        norm = F.conv2d(x ** 2, gamma, beta)
        norm = torch.sqrt(norm) if inverse else torch.rsqrt(norm)
        return x * norm

    def subpel(self, x, p):
        return F.pixel_shuffle(self.conv(x, p), 2)

    # -- residual blocks (res_blk.py) ------------------------------------------
    def rbws(self, x, p, dw):
        out = F.gelu(self.conv3x3(x, f"{p}.conv1", 2, dw))
        out = self.gdn(self.conv3x3(out, f"{p}.conv2", 1, dw), f"{p}.gdn", False)
        out += self.conv(x, f"{p}.skip", stride=2)
        return out

    def rb(self, x, p, dw):
        out = F.gelu(self.conv3x3(x, f"{p}.conv1", 1, dw))
        out = F.gelu(self.conv3x3(out, f"{p}.conv2", 1, dw))
        identity = self.conv(x, f"{p}.skip") if f"{p}.skip.weight" in self.sd else x
        return out + identity

    def rbu(self, x, p):
        out = F.gelu(self.subpel(x, f"{p}.subpel_conv.0"))
        out = self.gdn(self.dwsep(out, f"{p}.conv"), f"{p}.igdn", True)
        out += self.subpel(x, f"{p}.upsample.0")
        return out

    # -- transforms --------------------------------------------------------------
    def g_a(self, x):
        dw = not self.cfg.small_decoder
        g = "g_a.analysis_transform"
        x = self.rbws(x, f"{g}.0", dw)
        x = self.rb(x, f"{g}.1", dw)
        x = self.rbws(x, f"{g}.2", dw)
        x = self.rb(x, f"{g}.3", dw)
        x = self.rbws(x, f"{g}.4", dw)
        x = self.rb(x, f"{g}.5", dw)
        return self.conv3x3(x, f"{g}.6", 2, dw)

    def h_a(self, y):
        dw = not self.cfg.small_decoder
        h = "h_a.reduction"
        x = F.gelu(self.conv3x3(y, f"{h}.0", 1, dw))
        x = F.gelu(self.conv3x3(x, f"{h}.2", 1, dw))
        x = F.gelu(self.conv3x3(x, f"{h}.4", 2, dw))
        x = F.gelu(self.conv3x3(x, f"{h}.6", 1, dw))
        return self.conv3x3(x, f"{h}.8", 2, dw)

    def h_s(self, z):
        h = "h_s.increase"
        x = F.gelu(self.dwsep(z, f"{h}.0"))
        x = F.gelu(self.subpel(x, f"{h}.2.0"))
        x = F.gelu(self.dwsep(x, f"{h}.4"))
        x = F.gelu(self.subpel(x, f"{h}.6.0"))
        return self.dwsep(x, f"{h}.8")

    def g_s(self, y):
        g = "g_s.synthesis_transform"
        x = self.rb(y, f"{g}.0", True)
        x = self.rbu(x, f"{g}.1")
        x = self.rb(x, f"{g}.2", True)
        x = self.rbu(x, f"{g}.3")
        x = self.rb(x, f"{g}.4", True)
        x = self.rbu(x, f"{g}.5")
        x = self.rb(x, f"{g}.6", True)
        return self.subpel(x, f"{g}.7.0")

    # -- entropy bottleneck (compressai EntropyBottleneck, eval) ----------------
    def eb_medians(self):
        return self.sd["entropy_bottleneck.quantiles"][:, :, 1:2]   # [C,1,1]

    def eb_logits_cumulative(self, v):
        p = "entropy_bottleneck"
        logits = v
        for i in range(5):
            logits = torch.matmul(F.softplus(self.sd[f"{p}._matrix{i}"]), logits)
            logits = logits + self.sd[f"{p}._bias{i}"]
            if i < 4:
                logits = logits + torch.tanh(self.sd[f"{p}._factor{i}"]) * torch.tanh(logits)
        return logits

    def eb_likelihood(self, z):
        """z [B,C,h,w] -> likelihood of round(z - med) + med, bounded at 1e-9."""
        B, C, h, w = z.shape
        vals = z.permute(1, 0, 2, 3).reshape(C, 1, -1)
        med = self.eb_medians()
        out = torch.round(vals - med) + med
        lower = self.eb_logits_cumulative(out - 0.5)
        upper = self.eb_logits_cumulative(out + 0.5)
        lik = torch.sigmoid(upper) - torch.sigmoid(lower)
        lik = torch.max(lik, torch.tensor([1e-9], dtype=torch.float32))
        return lik.reshape(C, B, h, w).permute(1, 0, 2, 3).contiguous()

    # -- MEM++ context models (context.py) -----------------------------------------
    def local_context(self, x, i):
        """context.py:67-112."""
        p = f"local_context.{i}"
        B, C, H, W = x.shape
        L = H * W
        win = self.cfg.context_window
        heads, hd = 2, C // 2
        key = (H, W)
        if key not in self._mask_cache:
            self._mask_cache[key] = local_attn_mask(H, W, win)
        mask = self._mask_cache[key]
        t = x.reshape(B, C, L).permute(0, 2, 1)
        t = F.layer_norm(t, (C,), self.sd[f"{p}.norm1.weight"], self.sd[f"{p}.norm1.bias"], 1e-5)
        qkv = F.linear(t, self.sd[f"{p}.qkv_proj.weight"], self.sd[f"{p}.qkv_proj.bias"])
        qkv = qkv.reshape(B, H, W, 3, C).permute(3, 0, 4, 1, 2)
        qkv = torch.cat([qkv[0], qkv[1], qkv[2]], dim=1)
        wins = F.unfold(qkv, kernel_size=win, padding=(win - 1) // 2).permute(0, 2, 1)
        wins = wins.view(B, L, 3, C, win, win).permute(2, 0, 1, 3, 4, 5)

        def heads_split(t):   # channel c = d * heads + h  (interleaved)
            return t.reshape(B, L, hd, heads, win * win).permute(0, 1, 3, 4, 2)
        q, k, v = heads_split(wins[0]), heads_split(wins[1]), heads_split(wins[2])
        q = q * (hd ** -0.5)
        attn = q @ k.transpose(-2, -1)
        idx = self.sd[f"{p}.relative_position_index"].view(-1)
        bias = self.sd[f"{p}.relative_position_table"][idx].view(win * win, win * win, -1).permute(2, 0, 1)
        attn = attn + bias.unsqueeze(0).unsqueeze(1)
        attn = attn + mask.unsqueeze(0).unsqueeze(2)
        attn = torch.softmax(attn, dim=-1)
        o = (attn @ v).reshape(B, L, heads, win, win, hd).permute(0, 1, 3, 4, 2, 5)
        o = o.reshape(B * L, win, win, C).permute(0, 3, 1, 2)   # head-major merge: c = h * hd + d
        o = F.conv2d(o, self.sd[f"{p}.fusion.weight"], self.sd[f"{p}.fusion.bias"]).reshape(B, L, 2 * C)
        o = F.linear(o, self.sd[f"{p}.proj.weight"], self.sd[f"{p}.proj.bias"])
        n2 = F.layer_norm(o, (2 * C,), self.sd[f"{p}.norm2.weight"], self.sd[f"{p}.norm2.bias"], 1e-5)
        m = F.linear(F.gelu(F.linear(n2, self.sd[f"{p}.mlp.fc1.weight"], self.sd[f"{p}.mlp.fc1.bias"])),
                     self.sd[f"{p}.mlp.fc2.weight"], self.sd[f"{p}.mlp.fc2.bias"])
        o = o + m
        return o.permute(0, 2, 1).reshape(B, 2 * C, H, W)

    def channel_context(self, x, i):
        p = f"channel_context.{i}.fushion"
        dw = not self.cfg.small_decoder
        x = F.gelu(self.conv3x3(x, f"{p}.0", 1, dw))
        x = F.gelu(self.conv3x3(x, f"{p}.2", 1, dw))
        return self.conv3x3(x, f"{p}.4", 1, dw)

    def _qkv_branch(self, x, p):
        x = self.conv(x, f"{p}.0")
        return self.conv(x, f"{p}.1", groups=x.shape[1])

    @staticmethod
    def _linear_attention(keys, queries, values, heads):
        """ctx = softmax_L(K_h) V_h^T, out_h = ctx^T softmax_ch(Q_h)  (context.py:178-190, 233-242)."""
        B, D, _ = keys.shape
        hd = D // heads
        outs = []
        for h in range(heads):
            sl = slice(h * hd, (h + 1) * hd)
            k = F.softmax(keys[:, sl, :], dim=2)
            q = F.softmax(queries[:, sl, :], dim=1)
            ctx = k @ values[:, sl, :].transpose(1, 2)
            outs.append(ctx.transpose(1, 2) @ q)
        return torch.cat(outs, dim=1)

    def inter_context(self, x, i):
        """context.py:226-245."""
        p = f"global_inter_context.{i}"
        B, D, H, W = x.shape
        q = self._qkv_branch(x, f"{p}.queries").reshape(B, D, H * W)
        k = self._qkv_branch(x, f"{p}.keys").reshape(B, D, H * W)
        v = self._qkv_branch(x, f"{p}.values").reshape(B, D, H * W)
        heads = D // 32
        a = self._linear_attention(k, q, v, heads).reshape(B, D, H, W)
        a = self.conv(a, f"{p}.reprojection")
        m = F.gelu(self.conv(a, f"{p}.mlp.0"))
        m = F.gelu(self.conv(m, f"{p}.mlp.2", groups=m.shape[1]))
        m = self.conv(m, f"{p}.mlp.4")
        return self.conv(a, f"{p}.skip") + m

    def intra_context(self, x1, x2, i):
        """context.py:169-193: queries from non-anchor cells of x1, keys from anchor cells of
        x1, values from anchor cells of x2; softmaxes over the squeezed half grid."""
        p = f"global_intra_context.{i}"
        B, D, H, W = x1.shape
        q = ckbd_squeeze(self._qkv_branch(ckbd_nonanchor(x1), f"{p}.queries"), False)
        k = ckbd_squeeze(self._qkv_branch(ckbd_anchor(x1), f"{p}.keys"), True)
        v = ckbd_squeeze(self._qkv_branch(x2, f"{p}.values"), True)
        heads, hd = 2, D // 2
        outs = []
        for h in range(heads):
            sl = slice(h * hd, (h + 1) * hd)
            kh = F.softmax(k[:, sl].reshape(B, hd, -1), dim=2).reshape(B, hd, H, W // 2)
            qh = F.softmax(q[:, sl].reshape(B, hd, -1), dim=1).reshape(B, hd, H, W // 2)
            kh = ckbd_unsqueeze(kh, True).reshape(B, hd, H * W)
            vh = ckbd_unsqueeze(v[:, sl], True).reshape(B, hd, H * W)
            qh = ckbd_unsqueeze(qh, False).reshape(B, hd, H * W)
            ctx = kh @ vh.transpose(1, 2)
            outs.append((ctx.transpose(1, 2) @ qh).reshape(B, hd, H, W))
        a = self.conv(torch.cat(outs, dim=1), f"{p}.reprojection")
        m = F.gelu(self.conv(a, f"{p}.mlp.0"))
        m = F.gelu(self.conv(m, f"{p}.mlp.2", groups=m.shape[1]))
        return a + self.conv(m, f"{p}.mlp.4")

    def entropy_parameters(self, x, kind, i):
        p = f"entropy_parameters_{kind}.{i}.fusion"
        x = F.gelu(self.conv(x, f"{p}.0"))
        x = F.gelu(self.conv(x, f"{p}.2"))
        x = F.gelu(self.conv(x, f"{p}.4"))
        return self.conv(x, f"{p}.6")

    def lrp(self, x, kind, i):
        p = f"lrp_{kind}.{i}.lrp_transform"
        n = len(spec.lrp_dims(self.cfg, x.shape[1]))
        for j in range(n):
            x = self.dwsep(x, f"{p}.{2 * j}")
            if j < n - 1:
                x = F.gelu(x)
        return 0.5 * torch.tanh(x)

    # -- the slice loop -------------------------------------------------------------
    def _vbr_scale(self, s):
        if not self.cfg.vbr:
            return None
        g = self.sd["Gain"]
        s = max(0, min(int(s), len(g) - 1))
        return g[s]

    def _slice_loop(self, hyper, y=None, source=None, scale=None, record=None, collect_lik=True):
        """Runs the 10-slice MEM++ loop.  With y given it quantizes y (encoder / forward);
        with `source` it takes per-phase symbols from a callable (decoder).  `record(phase,
        symbols, indexes)` receives the coder streams in squeezed C-order."""
        cfg = self.cfg
        S, C = cfg.slice_num, cfg.slice_ch
        hM = cfg.hyper_M
        hyper_means = hyper[:, hM:]
        table = scale_table()
        rescale = None if scale is None else 1.0 / scale
        yh: List[T] = []
        liks: List[T] = []

        def quant(val, m):  # ste_round(val - m) + m  (VBR: ste_round((val - m) * sc) * resc + m)
            if scale is None:
                return torch.round(val - m) + m
            return torch.round((val - m) * scale) * rescale + m

        def phase(anchor, y_part, s_part, m_part, ph):
            if source is not None:
                s_sq = ckbd_squeeze(s_part, anchor)
                m_sq = ckbd_squeeze(m_part, anchor)
                idx = build_indexes(s_sq if scale is None else s_sq * scale, table)
                sym = source(ph, idx).reshape(s_sq.shape).float()
                val = sym + m_sq if scale is None else sym * rescale + m_sq
                return ckbd_unsqueeze(val, anchor)
            if record is not None:
                s_sq = ckbd_squeeze(s_part, anchor)
                m_sq = ckbd_squeeze(m_part, anchor)
                y_sq = ckbd_squeeze(y_part, anchor)
                idx = build_indexes(s_sq if scale is None else s_sq * scale, table)
                if scale is None:
                    sym = torch.round(y_sq - m_sq).int()
                else:
                    sym = torch.round((y_sq - m_sq) * scale).int()
                record(ph, sym, idx)
            return quant(y_part, m_part)

        for idx in range(S):
            y_slice = None if y is None else y[:, idx * C:(idx + 1) * C]
            ya = None if y is None else ckbd_anchor(y_slice)
            yn = None if y is None else ckbd_nonanchor(y_slice)
            if idx == 0:
                pa = self.entropy_parameters(hyper, "anchor", idx)
            else:
                prev = torch.cat(yh, dim=1)
                inter = self.inter_context(prev, idx)
                chan = self.channel_context(prev, idx)
                pa = self.entropy_parameters(torch.cat([inter, chan, hyper], dim=1), "anchor", idx)
            sa, ma = pa.chunk(2, 1)
            sa, ma = ckbd_anchor(sa), ckbd_anchor(ma)
            anc = phase(True, ya, sa, ma, 2 * idx)
            anc = anc + ckbd_anchor(self.lrp(torch.cat([hyper_means] + yh + [anc], dim=1), "anchor", idx))
            local = self.local_context(anc, idx)
            if idx == 0:
                pn = self.entropy_parameters(torch.cat([local, hyper], dim=1), "nonanchor", idx)
            else:
                intra = self.intra_context(yh[-1], anc, idx)
                pn = self.entropy_parameters(torch.cat([local, intra, inter, chan, hyper], dim=1), "nonanchor", idx)
            sn, mn = pn.chunk(2, 1)
            sn, mn = ckbd_nonanchor(sn), ckbd_nonanchor(mn)
            if y is not None and collect_lik:
                s_all, m_all = sa + sn, ma + mn
                if scale is None:
                    liks.append(gaussian_likelihood(y_slice, s_all, m_all))
                else:
                    liks.append(gaussian_likelihood(y_slice * scale, s_all * scale, m_all * scale))
            non = phase(False, yn, sn, mn, 2 * idx + 1)
            cur = anc + non
            cur = cur + ckbd_nonanchor(self.lrp(torch.cat([hyper_means] + yh + [cur], dim=1), "nonanchor", idx))
            yh.append(cur)
        return torch.cat(yh, dim=1), (torch.cat(liks, dim=1) if liks else None)

    # -- public entry points ------------------------------------------------------------
    @torch.no_grad()
    def forward(self, x, s: int = 1):
        """mlicpp.py:79-185 (VBR: stage 2, Gain[s])."""
        scale = self._vbr_scale(s)
        y = self.g_a(x)
        z = self.h_a(y)
        z_lik = self.eb_likelihood(z)
        med = self.eb_medians()
        z_hat = torch.round(z - med) + med
        hyper = self.h_s(z_hat)
        y_hat, y_lik = self._slice_loop(hyper, y=y, scale=scale)
        x_hat = self.g_s(y_hat)
        return {"x_hat": x_hat, "likelihoods": {"y_likelihoods": y_lik, "z_likelihoods": z_lik},
                "y_hat": y_hat}

    @torch.no_grad()
    def compress_streams(self, x, s: int = 1, likelihoods: bool = False):
        """Encoder side of mlicpp.py:199-290 minus the rANS coder: returns the z symbols
        (round(z - median), int32 [B,C,h,w]) and the 20 per-phase (symbols, indexes) int32
        arrays in the exact order BufferedRansEncoder receives them, plus y_hat.  likelihoods=True
        also returns the y / z likelihoods of the same pass (forward's, mlicpp.py:140-185), so
        bpp_lik comes with the streams at no second network pass."""
        scale = self._vbr_scale(s)
        y = self.g_a(x)
        z = self.h_a(y)
        med = self.eb_medians()
        z_sym = torch.round(z - med.reshape(1, -1, 1, 1)).int()
        z_hat = z_sym.float() + med.reshape(1, -1, 1, 1)
        hyper = self.h_s(z_hat)
        streams = {}

        def record(ph, sym, idx):
            streams[ph] = (sym.clone(), idx.clone())
        y_hat, y_lik = self._slice_loop(hyper, y=y, scale=scale, record=record, collect_lik=likelihoods)
        out = {"z_symbols": z_sym, "phases": [streams[k] for k in sorted(streams)], "y_hat": y_hat,
               "z_hat": z_hat}
        if likelihoods:
            out["likelihoods"] = {"y_likelihoods": y_lik, "z_likelihoods": self.eb_likelihood(z)}
        return out

    @torch.no_grad()
    def decode_streams(self, z_symbols, phase_symbols, s: int = 1):
        """Decoder side of mlicpp.py:292-378 given the decoded integer streams."""
        scale = self._vbr_scale(s)
        med = self.eb_medians().reshape(1, -1, 1, 1)
        z_hat = z_symbols.float() + med
        hyper = self.h_s(z_hat)

        def source(ph, idx):
            return phase_symbols[ph]
        y_hat, _ = self._slice_loop(hyper, source=source, scale=scale)
        return {"x_hat": self.g_s(y_hat), "y_hat": y_hat}


def bpp_from_likelihoods(y_lik: T, z_lik: T, num_pixels: int) -> float:
    """loss/rd_loss.py:42-45."""
    return float(sum(torch.log(l).sum() / (-math.log(2) * num_pixels) for l in (y_lik, z_lik)))


def psnr_uint8(a: T, b: T) -> float:
    """utils/utils.py:86-87 torch2img (clamp, *255, truncate) + utils/metrics.py:32-33."""
    def to_u8(t):
        return (t.clamp(0, 1) * 255).to(torch.uint8).float()
    mse = torch.mean((to_u8(a) - to_u8(b)) ** 2).item()
    return 20 * math.log10(255.0) - 10 * math.log10(mse) if mse > 0 else float("inf")
