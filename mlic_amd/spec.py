"""Model configurations and the state_dict inventory of the MLIC++ family.

The drop-in contract is "same state_dict keys and shapes as the reference":
a checkpoint trained with LuZWCHA/MLIC loads into this package unchanged.
This module restates, from the reference's module tree, the name and shape of
every parameter and buffer, per model variant:

* configs ............ MLIC++/config/config.py:19-62 (model_config)
* factory names ...... MLIC++/models/model_loader.py:4-18 (get_model)
* MLICPlusPlus ....... MLIC++/models/mlicpp.py:14-77
* MLICPlusPlusSD ..... MLIC++/models/mlicpp_small_decoder.py:16-83
* MLICPlusPlusVbr .... MLIC++/models/mlicpp_vbr.py:14-120
* MLICPlusPlusSDVbr .. MLIC++/models/mlicpp_sd_vbr.py:19-118 (the small-decoder tree + the VBR gains)
* layer naming ....... MLIC++/modules/layers/{conv,res_blk,attention}.py,
                       MLIC++/modules/transform/*.py, compressai 1.2.6 layers

Nothing here touches a GPU; the HIP executor and the weight packer both read
this inventory.
"""
from __future__ import annotations

import dataclasses
from collections import OrderedDict
from typing import Dict, Tuple

Shape = Tuple[int, ...]


@dataclasses.dataclass(frozen=True)
class ModelConfig:
    name: str
    N: int
    M: int
    slice_num: int
    context_window: int = 5
    # variant flags
    small_decoder: bool = False    # MLICPlusPlusSD (full-conv encoder, N/4 g_s, M/4 h_s)
    vbr: bool = False              # MLICPlusPlusVbr (Gain / QuantABCD)

    @property
    def slice_ch(self) -> int:
        return self.M // self.slice_num

    @property
    def hyper_M(self) -> int:
        """Channel count of hyper_means (= half of h_s output)."""
        return self.M // 4 if self.small_decoder else self.M

    @property
    def gs_N(self) -> int:
        return self.N // 4 if self.small_decoder else self.N


# config/config.py:19-62. MLICPP_L_VBR is not registered in the reference
# (config.py falls through to an unbound name); SURVEY §5 asks for it with
# MLICPP_L dims, which is what we register.
CONFIGS: Dict[str, ModelConfig] = {
    "MLICPP_L": ModelConfig("MLICPP_L", 192, 320, 10),
    "MLICPP_S": ModelConfig("MLICPP_S", 96, 160, 5),
    "MLICPP_S_VBR": ModelConfig("MLICPP_S_VBR", 96, 160, 5, vbr=True),
    "MLICPP_L_VBR": ModelConfig("MLICPP_L_VBR", 192, 320, 10, vbr=True),
    "MLICPP_M": ModelConfig("MLICPP_M", 160, 256, 8),
    "MLICPP_S2": ModelConfig("MLICPP_S2", 128, 128, 2),
    "MLICPP_M_SMALL_DEC": ModelConfig("MLICPP_M_SMALL_DEC", 192, 320, 10, small_decoder=True),
    # models/model_loader.py:14-15, config/config.py:52-59 (the MLICPP_M_SMALL_DEC dimensions)
    "MLICPP_M_SMALL_DEC_VBR": ModelConfig("MLICPP_M_SMALL_DEC_VBR", 192, 320, 10, small_decoder=True, vbr=True),
}

# VBR constants, mlicpp_vbr.py:83-91
VBR_LAMBDAS = (0.0005, 0.0035, 0.0067, 0.025, 0.0483, 0.18)
VBR_GAIN = (0.06556, 0.13944, 0.19293, 0.37268, 0.51801, 1.00000)
# the small-decoder VBR model's five levels, mlicpp_sd_vbr.py:89-97
SD_VBR_LAMBDAS = (0.0002, 0.0005, 0.0035, 0.0483, 0.18)
SD_VBR_GAIN = (0.002424, 0.06556, 0.13944, 0.51801, 1.00000)


def vbr_lambdas(name: str) -> Tuple[float, ...]:
    cfg = get_config(name)
    return SD_VBR_LAMBDAS if cfg.small_decoder else VBR_LAMBDAS


def vbr_gain(name: str) -> Tuple[float, ...]:
    """The Gain parameter's initial value (= its trained size) of a VBR model."""
    cfg = get_config(name)
    return SD_VBR_GAIN if cfg.small_decoder else VBR_GAIN


def get_config(name: str) -> ModelConfig:
    try:
        return CONFIGS[name]
    except KeyError:
        raise ValueError(f"unknown model name {name!r}; known: {sorted(CONFIGS)}") from None


class _Inv:
    """Accumulates (key -> shape) in module-registration order."""

    def __init__(self):
        self.d: "OrderedDict[str, Shape]" = OrderedDict()

    def add(self, key: str, shape: Shape):
        assert key not in self.d, key
        self.d[key] = tuple(int(s) for s in shape)

    # --- layer vocab -------------------------------------------------------
    def conv(self, p: str, cin: int, cout: int, k: int, groups: int = 1, bias: bool = True):
        self.add(f"{p}.weight", (cout, cin // groups, k, k))
        if bias:
            self.add(f"{p}.bias", (cout,))

    def linear(self, p: str, cin: int, cout: int):
        self.add(f"{p}.weight", (cout, cin))
        self.add(f"{p}.bias", (cout,))

    def dwsep(self, p: str, cin: int, cout: int):
        # modules/layers/conv.py:46-63 DepthWiseConv
        self.conv(f"{p}.depth_conv", cin, cin, 3, groups=cin)
        self.conv(f"{p}.point_conv", cin, cout, 1)

    def conv3x3(self, p: str, cin: int, cout: int, dw: bool):
        # modules/layers/conv.py:22-32: depthwise-separable by default in this fork
        if dw:
            self.dwsep(p, cin, cout)
        else:
            self.conv(p, cin, cout, 3)

    def gdn(self, p: str, c: int):
        # compressai GDN + NonNegativeParametrizer (params, then child buffers)
        self.add(f"{p}.beta", (c,))
        self.add(f"{p}.gamma", (c, c))
        self.add(f"{p}.beta_reparam.pedestal", (1,))
        self.add(f"{p}.beta_reparam.lower_bound.bound", (1,))
        self.add(f"{p}.gamma_reparam.pedestal", (1,))
        self.add(f"{p}.gamma_reparam.lower_bound.bound", (1,))

    def rbws(self, p: str, cin: int, cout: int, dw: bool):
        # res_blk.py:62-93 ResidualBlockWithStride (stride 2)
        self.conv3x3(f"{p}.conv1", cin, cout, dw)
        self.conv3x3(f"{p}.conv2", cout, cout, dw)
        self.gdn(f"{p}.gdn", cout)
        self.conv(f"{p}.skip", cin, cout, 1)

    def rb(self, p: str, cin: int, cout: int, dw: bool):
        # res_blk.py:124-154 ResidualBlock
        self.conv3x3(f"{p}.conv1", cin, cout, dw)
        self.conv3x3(f"{p}.conv2", cout, cout, dw)
        if cin != cout:
            self.conv(f"{p}.skip", cin, cout, 1)

    def rbu(self, p: str, cin: int, cout: int):
        # res_blk.py:96-121 ResidualBlockUpsample, subpel_conv3x3 = Sequential(conv, PixelShuffle)
        self.conv(f"{p}.subpel_conv.0", cin, cout * 4, 3)
        self.dwsep(f"{p}.conv", cout, cout)
        self.gdn(f"{p}.igdn", cout)
        self.conv(f"{p}.upsample.0", cin, cout * 4, 3)


def _entropy_bottleneck(inv: _Inv, N: int):
    # compressai EntropyBottleneck(N), filters (3,3,3,3)
    p = "entropy_bottleneck"
    inv.add(f"{p}._offset", (0,))            # buffers from EntropyModel (filled by update())
    inv.add(f"{p}._quantized_cdf", (0,))
    inv.add(f"{p}._cdf_length", (0,))
    inv.add(f"{p}.likelihood_lower_bound.bound", (1,))
    f = (1, 3, 3, 3, 3, 1)
    for i in range(5):
        inv.add(f"{p}._matrix{i}", (N, f[i + 1], f[i]))
        inv.add(f"{p}._bias{i}", (N, f[i + 1], 1))
        if i < 4:
            inv.add(f"{p}._factor{i}", (N, f[i + 1], 1))
    inv.add(f"{p}.quantiles", (N, 1, 3))
    inv.add(f"{p}.target", (3,))


def _gaussian_conditional(inv: _Inv):
    p = "gaussian_conditional"
    inv.add(f"{p}._offset", (0,))
    inv.add(f"{p}._quantized_cdf", (0,))
    inv.add(f"{p}._cdf_length", (0,))
    inv.add(f"{p}.likelihood_lower_bound.bound", (1,))
    inv.add(f"{p}.lower_bound_scale.bound", (1,))
    inv.add(f"{p}.scale_table", (0,))
    inv.add(f"{p}.scale_bound", (1,))


DYNAMIC_BUFFERS = ("_offset", "_quantized_cdf", "_cdf_length", "scale_table")


def state_dict_shapes(name: str) -> "OrderedDict[str, Shape]":
    """Every state_dict key of model `name` with its shape (dynamic CDF buffers
    are listed with their pre-update() shape)."""
    cfg = get_config(name)
    inv = _Inv()
    N, M, S, C = cfg.N, cfg.M, cfg.slice_num, cfg.slice_ch
    _entropy_bottleneck(inv, N)

    enc_dw = not cfg.small_decoder   # SD encoder uses analysis_old (full conv)
    # g_a  analysis.py:6-22
    g = "g_a.analysis_transform"
    inv.rbws(f"{g}.0", 3, N, enc_dw)
    inv.rb(f"{g}.1", N, N, enc_dw)
    inv.rbws(f"{g}.2", N, N, enc_dw)
    inv.rb(f"{g}.3", N, N, enc_dw)
    inv.rbws(f"{g}.4", N, N, enc_dw)
    inv.rb(f"{g}.5", N, N, enc_dw)
    inv.conv3x3(f"{g}.6", N, M, enc_dw)
    # h_a  analysis.py:25-48 (VBR registers g_s before h_a; order is irrelevant for loading)
    h = "h_a.reduction"
    inv.conv3x3(f"{h}.0", M, N, enc_dw)
    inv.conv3x3(f"{h}.2", N, N, enc_dw)
    inv.conv3x3(f"{h}.4", N, N, enc_dw)
    inv.conv3x3(f"{h}.6", N, N, enc_dw)
    inv.conv3x3(f"{h}.8", N, N, enc_dw)
    # g_s  synthesis.py:56-73
    gN = cfg.gs_N
    g = "g_s.synthesis_transform"
    inv.rb(f"{g}.0", M, M, True)
    inv.rbu(f"{g}.1", M, gN)
    inv.rb(f"{g}.2", gN, gN, True)
    inv.rbu(f"{g}.3", gN, gN)
    inv.rb(f"{g}.4", gN, gN, True)
    inv.rbu(f"{g}.5", gN, gN)
    inv.rb(f"{g}.6", gN, gN, True)
    inv.conv(f"{g}.7.0", gN, 3 * 4, 3)
    # h_s  synthesis.py:9-33 (SD: HyperSynthesis(M=M//4, N=N))
    hM = cfg.hyper_M
    h = "h_s.increase"
    inv.dwsep(f"{h}.0", N, hM)
    inv.conv(f"{h}.2.0", hM, hM * 4, 3)
    inv.dwsep(f"{h}.4", hM, hM * 3 // 2)
    inv.conv(f"{h}.6.0", hM * 3 // 2, hM * 3 // 2 * 4, 3)
    inv.dwsep(f"{h}.8", hM * 3 // 2, hM * 2)
    _gaussian_conditional(inv)

    # MEM++ context models  context.py
    for i in range(S):
        p = f"local_context.{i}"
        inv.add(f"{p}.relative_position_table", ((2 * cfg.context_window - 1) ** 2, 2))
        inv.linear(f"{p}.qkv_proj", C, 3 * C)
        inv.linear(f"{p}.proj", 2 * C, 2 * C)
        inv.linear(f"{p}.mlp.fc1", 2 * C, 4 * C)
        inv.linear(f"{p}.mlp.fc2", 4 * C, 2 * C)
        inv.add(f"{p}.norm1.weight", (C,))
        inv.add(f"{p}.norm1.bias", (C,))
        inv.add(f"{p}.norm2.weight", (2 * C,))
        inv.add(f"{p}.norm2.bias", (2 * C,))
        inv.add(f"{p}.relative_position_index", (cfg.context_window ** 2, cfg.context_window ** 2))
        inv.conv(f"{p}.fusion", C, 2 * C, cfg.context_window)
    hidden = (96, 96) if cfg.small_decoder else (192, 128)
    chan_dw = not cfg.small_decoder  # SD uses context_old.ChannelContext (full conv)
    for i in range(1, S):
        p = f"channel_context.{i}.fushion"
        inv.conv3x3(f"{p}.0", C * i, hidden[0], chan_dw)
        inv.conv3x3(f"{p}.2", hidden[0], hidden[1], chan_dw)
        inv.conv3x3(f"{p}.4", hidden[1], C * 4, chan_dw)
    for i in range(1, S):
        p = f"global_inter_context.{i}"
        dim, out = C * i, C * 2
        for t in ("keys", "queries", "values"):
            inv.conv(f"{p}.{t}.0", dim, dim, 1)
            inv.conv(f"{p}.{t}.1", dim, dim, 3, groups=dim)
        inv.conv(f"{p}.reprojection", dim, out * 3 // 2, 5)
        inv.conv(f"{p}.mlp.0", out * 3 // 2, out * 2, 1)
        inv.conv(f"{p}.mlp.2", out * 2, out * 2, 3, groups=out * 2)
        inv.conv(f"{p}.mlp.4", out * 2, out, 1)
        inv.conv(f"{p}.skip", out * 3 // 2, out, 1)
    for i in range(1, S):
        p = f"global_intra_context.{i}"
        dim = C
        for t in ("keys", "queries", "values"):
            inv.conv(f"{p}.{t}.0", dim, dim, 1)
            inv.conv(f"{p}.{t}.1", dim, dim, 3, groups=dim)
        inv.conv(f"{p}.reprojection", dim, dim * 2, 5)
        inv.conv(f"{p}.mlp.0", dim * 2, dim * 4, 1)
        inv.conv(f"{p}.mlp.2", dim * 4, dim * 4, 3, groups=dim * 4)
        inv.conv(f"{p}.mlp.4", dim * 4, dim * 2, 1)
    # entropy.py:7-29 EntropyParameters; in_dims from mlicpp.py:57-66 with M -> hyper_M for SD
    hp = 2 * hM
    for kind, first, rest in (("anchor", hp, hp + C * 6), ("nonanchor", hp + C * 2, hp + C * 10)):
        for i in range(S):
            p = f"entropy_parameters_{kind}.{i}.fusion"
            cin = first if i == 0 else rest
            inv.conv(f"{p}.0", cin, 320, 1)
            inv.conv(f"{p}.2", 320, 256, 1)
            inv.conv(f"{p}.4", 256, 128, 1)
            inv.conv(f"{p}.6", 128, C * 2, 1)
    # quantization.py LatentResidualPrediction(Old)
    for kind in ("anchor", "nonanchor"):
        for i in range(S):
            p = f"lrp_{kind}.{i}.lrp_transform"
            cin = hM + (i + 1) * C
            for j, (a, b) in enumerate(lrp_dims(cfg, cin)):
                inv.dwsep(f"{p}.{2 * j}", a, b)
    if cfg.vbr:
        inv.add("Gain", (len(vbr_gain(name)),))
        inv.linear("QuantABCD.0", 2, 12)
        inv.linear("QuantABCD.2", 12, 12)
        inv.linear("QuantABCD.4", 12, 1)
    return inv.d


def lrp_dims(cfg: ModelConfig, cin: int):
    """(in, out) channel pairs of the LRP conv chain (quantization.py:9-44)."""
    C = cfg.slice_ch
    if cfg.small_decoder:
        diff = abs(C - cin)
        chans = [cin, cin - diff // 4, cin - diff // 2, cin - diff * 3 // 4, C]
    else:
        chans = [cin, 224, 128, C]
    return list(zip(chans[:-1], chans[1:]))


def param_count(name: str) -> int:
    n = 0
    for k, s in state_dict_shapes(name).items():
        leaf = k.rsplit(".", 1)[-1]
        if leaf in DYNAMIC_BUFFERS or leaf in ("pedestal", "bound", "target", "scale_bound",
                                                "relative_position_index"):
            continue
        c = 1
        for d in s:
            c *= d
        n += c
    return n
