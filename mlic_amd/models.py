"""Drop-in MLIC++ models: the reference's CompressionModel API over the HIP executor.

    net = get_model("MLICPP_L")             # models/model_loader.py:4-18
    net.load_state_dict(ckpt["state_dict"])  # same keys and shapes as the reference
    net = net.cuda().eval()
    out = net(x)                             # {"x_hat", "likelihoods": {"y_likelihoods", "z_likelihoods"}}
    net.update()
    c = net.compress(x)                      # {"strings": [[y], [z...]], "shape", "cost_time"}
    d = net.decompress(c["strings"], c["shape"])

The module holds the state_dict tensors under the reference's names (nested container modules,
so `state_dict()` / `load_state_dict()` / `.to()` / `parameters()` behave as in the reference).
All compute runs in libmlic_hip.so on the tensors' HIP device; there is no CPU path: calling the
model with CPU tensors raises.
"""
from __future__ import annotations

import ctypes as C
import time
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn as nn

from . import _lib, entropy, spec

_BUFFER_LEAVES = {"pedestal", "bound", "target", "scale_bound", "relative_position_index", "_offset",
                  "_quantized_cdf", "_cdf_length", "scale_table"}


class _Node(nn.Module):
    """Container module used only to reproduce the reference's dotted state_dict names."""


def _child(root: nn.Module, path: List[str]) -> nn.Module:
    m = root
    for part in path:
        if part not in m._modules:
            m.add_module(part, _Node())
        m = m._modules[part]
    return m


class MLICPlusPlus(nn.Module):
    """MLIC++ (models/mlicpp.py:13-475) with the hot path in HIP."""

    def __init__(self, config=None, name: str = "MLICPP_L", **kwargs):
        super().__init__()
        if config is not None and hasattr(config, "name"):
            name = config.name
        self.cfg = spec.get_config(name)
        self.model_name = name
        self.N, self.M = self.cfg.N, self.cfg.M
        self.slice_num, self.slice_ch = self.cfg.slice_num, self.cfg.slice_ch
        self.context_window = self.cfg.context_window
        from .synthetic import synth_state_dict  # default init = the seeded conditioned set
        sd = synth_state_dict(name, seed=0)
        for key, t in sd.items():
            *path, leaf = key.split(".")
            owner = _child(self, path)
            if leaf in _BUFFER_LEAVES:
                owner.register_buffer(leaf, t.clone())
            else:
                owner.register_parameter(leaf, nn.Parameter(t.clone(), requires_grad=False))
        self._handle = None
        self._handle_key = None
        self._tables_pushed = None

    # ---------------------------------------------------------------- state
    def load_state_dict(self, state_dict, strict: bool = True):
        """mlicpp.py:461-468: resize the dynamic CDF buffers, then load."""
        for key, val in state_dict.items():
            *path, leaf = key.split(".")
            if leaf in spec.DYNAMIC_BUFFERS:
                owner = _child(self, path)
                if leaf in owner._buffers:
                    owner._buffers[leaf] = torch.empty_like(val, device=owner._buffers[leaf].device)
        res = super().load_state_dict(state_dict, strict=strict)
        self._invalidate()
        return res

    def _apply(self, fn, *a, **k):
        out = super()._apply(fn, *a, **k)
        self._invalidate()
        return out

    def _invalidate(self):
        self._handle_key = None
        self._tables_pushed = None

    def __del__(self):
        try:
            self._release()
        except Exception:
            pass

    def _release(self):
        if getattr(self, "_handle", None) is not None:
            _lib.lib().mlic_destroy(self._handle)
            self._handle = None

    @property
    def device(self) -> torch.device:
        return self.g_a.analysis_transform._modules["0"].skip.weight.device

    def _weights(self):
        """(names, tensors) of every float tensor the executor needs, on the model's device."""
        names, tensors = [], []
        for k, v in self.state_dict().items():
            if v.dtype != torch.float32 or v.numel() == 0:
                continue
            if k.rsplit(".", 1)[-1] in ("scale_table",):
                continue
            names.append(k)
            tensors.append(v.detach().contiguous())
        names.append("__scale_table")
        tensors.append(entropy.get_scale_table().to(self.device))
        return names, tensors

    def _ensure_handle(self, dev: torch.device):
        if dev.type != "cuda":
            raise RuntimeError("mlic_amd runs only on a HIP device (MI355X); got tensors on " + str(dev))
        if self.device != dev:
            raise RuntimeError(f"model weights are on {self.device}, input on {dev}")
        key = (str(dev),)
        if self._handle is not None and self._handle_key == key:
            return self._handle
        self._release()
        names, tensors = self._weights()
        n = len(names)
        arr_names = (C.c_char_p * n)(*[s.encode() for s in names])
        arr_ptrs = (C.c_void_p * n)(*[t.data_ptr() for t in tensors])
        shapes = np.ones((n, 4), np.int64)
        ndims = np.zeros(n, np.int32)
        for i, t in enumerate(tensors):
            ndims[i] = t.dim()
            shapes[i, : t.dim()] = list(t.shape)
        h = C.c_void_p()
        with torch.cuda.device(dev):
            stream = torch.cuda.current_stream().cuda_stream
            _lib.call("mlic_create", self.model_name.encode(), n, arr_names, arr_ptrs,
                      shapes.ctypes.data_as(C.POINTER(C.c_int64)), ndims.ctypes.data_as(C.POINTER(C.c_int)),
                      C.c_void_p(stream), C.byref(h))
        self._handle = h
        self._handle_key = key
        self._tables_pushed = None
        if getattr(self, "_lanes", None):
            _lib.call("mlic_set_lanes", h, self._lanes)
        if getattr(self, "_prio_base", None):
            _lib.call("mlic_set_priority_base", h, self._prio_base)
        if getattr(self, "_precision", None) is not None:
            _lib.call("mlic_set_precision", h, self._precision)
        if getattr(self, "_synth_precision", None) is not None:
            _lib.call("mlic_set_synthesis_precision", h, self._synth_precision)
        return h

    def _vbr_scales(self, B: int, **kw) -> np.ndarray:
        """Per-image VBR gain (float32 [B]); 1 for fixed-rate models."""
        return np.ones(B, np.float32)

    def set_precision(self, mode: int):
        """Dense-conv arithmetic: 2 = split-fp16 MFMA "f16x3" (default), 0 = fp32 MFMA."""
        self._precision = int(mode)
        if self._handle is not None:
            _lib.call("mlic_set_precision", self._handle, self._precision)

    def set_synthesis_precision(self, mode: int):
        """g_s only (synthesis.py:56-73): 0 = the model precision (default), 1 = its dense subpel convs on
        fp16 operands with fp32 accumulation.  x_hat changes within the 0.01 dB gate; bitstreams do not."""
        self._synth_precision = int(mode)
        if self._handle is not None:
            _lib.call("mlic_set_synthesis_precision", self._handle, self._synth_precision)

    def set_priority_base(self, base: int):
        """Stream-priority offset of this model's lanes (scheduling only; set before the first call)."""
        self._prio_base = int(base)
        if self._handle is not None:
            _lib.call("mlic_set_priority_base", self._handle, self._prio_base)

    def set_lanes(self, n: int):
        """Host threads x HIP streams used by compress()/decompress() (results do not depend on it)."""
        self._lanes = int(n)
        if self._handle is not None:
            _lib.call("mlic_set_lanes", self._handle, self._lanes)

    @staticmethod
    def _out(shape, dev):
        """An output buffer: uninitialised, or NaN under the $MLIC_POISON test switch (an element the
        library does not write then fails every equality and finiteness check)."""
        if _lib.poison():
            return torch.full(tuple(shape), float("nan"), device=dev)
        return torch.empty(tuple(shape), device=dev)

    def range_fallbacks(self, reset: bool = False) -> Dict[str, int]:
        """fp16 range-guard fallbacks taken by this model since the last reset (mlic_range_fallbacks):
        forward re-run whole in exact fp32, forward's g_s alone, decompress's g_s alone."""
        if self._handle is None:
            return {"forward_full": 0, "forward_gs": 0, "decompress_gs": 0}
        a, b, c = C.c_int64(), C.c_int64(), C.c_int64()
        _lib.call("mlic_range_fallbacks", self._handle, C.byref(a), C.byref(b), C.byref(c), int(reset))
        return {"forward_full": a.value, "forward_gs": b.value, "decompress_gs": c.value}

    @staticmethod
    def _stream():
        return C.c_void_p(torch.cuda.current_stream().cuda_stream)

    # ---------------------------------------------------------------- API
    def update_resolutions(self, H, W, device=None):
        """mlicpp.py:187-197.  The HIP attention derives its checkerboard mask from parity bits, so
        there is no per-resolution mask tensor to rebuild; kept for API compatibility."""
        return False

    @torch.no_grad()
    def forward(self, x: torch.Tensor, **kw):
        """mlicpp.py:79-185."""
        if x.dim() != 4 or x.size(1) != 3:
            raise ValueError(f"expected [B,3,H,W], got {tuple(x.shape)}")
        B, _, H, W = x.shape
        if H % 64 or W % 64:
            raise ValueError("H and W must be multiples of 64 (pad as utils/testing.py:130-137)")
        h = self._ensure_handle(x.device)
        x = x.contiguous().float()
        x_hat = self._out(x.shape, x.device)
        y_lik = self._out((B, self.M, H // 16, W // 16), x.device)
        z_lik = self._out((B, self.N, H // 64, W // 64), x.device)
        sc = self._vbr_scales(B, **kw)
        _lib.call("mlic_forward_v", h, self._stream(), x.data_ptr(), B, H, W, x_hat.data_ptr(), y_lik.data_ptr(),
                  z_lik.data_ptr(), sc.ctypes.data)
        return {"x_hat": x_hat, "likelihoods": {"y_likelihoods": y_lik, "z_likelihoods": z_lik}}

    def update(self, scale_table=None, force: bool = False) -> bool:
        """mlicpp.py:470-475: build the GaussianConditional (64 scales) and EntropyBottleneck CDFs."""
        gc = self.gaussian_conditional
        eb = self.entropy_bottleneck
        updated = False
        if gc._buffers["_offset"].numel() == 0 or force:
            st = entropy.get_scale_table() if scale_table is None else scale_table
            cdf, length, offset, st = entropy.gaussian_tables(st)
            dev = gc._buffers["_offset"].device
            gc._buffers["_quantized_cdf"] = cdf.to(dev)
            gc._buffers["_cdf_length"] = length.to(dev)
            gc._buffers["_offset"] = offset.to(dev)
            gc._buffers["scale_table"] = st.to(dev)
            updated = True
        if eb._buffers["_offset"].numel() == 0 or force:
            params = {k: v for k, v in eb._parameters.items()}
            cdf, length, offset = entropy.bottleneck_tables(params)
            dev = eb._buffers["_offset"].device
            eb._buffers["_quantized_cdf"] = cdf.to(dev)
            eb._buffers["_cdf_length"] = length.to(dev)
            eb._buffers["_offset"] = offset.to(dev)
            updated = True
        self._tables_pushed = None
        return updated

    def _push_tables(self, h):
        if self._tables_pushed is h:
            return
        gc, eb = self.gaussian_conditional, self.entropy_bottleneck
        if gc._buffers["_offset"].numel() == 0 or eb._buffers["_offset"].numel() == 0:
            raise RuntimeError("entropy tables are empty: call update() (or load a state_dict that has them)")
        keep = []

        def arr(t):
            a = np.ascontiguousarray(t.detach().cpu().numpy().astype(np.int32))
            keep.append(a)
            return a.ctypes.data
        g_cdf, e_cdf = gc._buffers["_quantized_cdf"], eb._buffers["_quantized_cdf"]
        _lib.call("mlic_set_entropy_tables", h,
                  arr(g_cdf), arr(gc._buffers["_cdf_length"].reshape(-1)), arr(gc._buffers["_offset"].reshape(-1)),
                  g_cdf.shape[0], g_cdf.shape[1],
                  arr(e_cdf), arr(eb._buffers["_cdf_length"].reshape(-1)), arr(eb._buffers["_offset"].reshape(-1)),
                  e_cdf.shape[0], e_cdf.shape[1])
        self._tables_pushed = h

    @torch.no_grad()
    def compress(self, x: torch.Tensor, batch_stream: bool = False, **kw):
        """mlicpp.py:199-290.  strings = [[y_stream per image], [z_stream per image]] (B = 1: exactly
        the reference's layout; for B > 1 each image gets its own y stream, which the host codes in
        parallel).  batch_stream=True: the reference's B > 1 layout instead, ONE y stream for the batch
        (mlicpp.py:215, 279-281; phase-major, image-minor).  decompress() accepts both.
        cost_time brackets the call with the caller's stream synchronised (the reference synchronises the
        whole device, mlicpp.py:200, 282; a stream keeps concurrent callers on other streams apart)."""
        torch.cuda.current_stream(x.device).synchronize()
        t0 = time.time()
        B, _, H, W = x.shape
        if H % 64 or W % 64:
            raise ValueError("H and W must be multiples of 64")
        h = self._ensure_handle(x.device)
        self._push_tables(h)
        x = x.contiguous().float()
        sc = self._vbr_scales(B, **kw)
        _lib.call("mlic_compress_v", h, self._stream(), x.data_ptr(), B, H, W, sc.ctypes.data)
        ys, zs = [], []
        for b in range(B):
            yl, zl = C.c_size_t(), C.c_size_t()
            _lib.call("mlic_encoded_size", h, b, C.byref(yl), C.byref(zl))
            yb = C.create_string_buffer(max(1, yl.value))
            zb = C.create_string_buffer(max(1, zl.value))
            _lib.call("mlic_encoded_copy", h, b, yb, zb)
            ys.append(C.string_at(yb, yl.value))
            zs.append(C.string_at(zb, zl.value))
        if batch_stream and B > 1:
            n = C.c_size_t()
            _lib.call("mlic_batch_stream", h, 0, B, None, 0, C.byref(n))
            buf = C.create_string_buffer(max(1, n.value))
            _lib.call("mlic_batch_stream", h, 0, B, buf, n.value, C.byref(n))
            ys = [C.string_at(buf, n.value)]
        torch.cuda.current_stream(x.device).synchronize()
        return {"strings": [ys, zs], "shape": torch.Size([H // 64, W // 64]), "cost_time": time.time() - t0}

    @torch.no_grad()
    def decompress(self, strings, shape, **kw):
        """mlicpp.py:292-378."""
        dev = self.device
        torch.cuda.current_stream(dev).synchronize()
        t0 = time.time()
        ys, zs = list(strings[0]), list(strings[1])
        B = len(zs)
        single = len(ys) == 1 and B > 1  # the reference's batched layout (mlicpp.py:306-307)
        if len(ys) != B and not single:
            raise ValueError("expected one y stream per image, or one stream for the whole batch")
        hz, wz = int(shape[0]), int(shape[1])
        h = self._ensure_handle(dev)
        self._push_tables(h)
        x_hat = self._out((B, 3, hz * 64, wz * 64), dev)
        ybufs = [C.create_string_buffer(s, len(s)) for s in ys]
        zbufs = [C.create_string_buffer(s, len(s)) for s in zs]
        yp = (C.c_void_p * B)(*[C.cast(b, C.c_void_p) for b in ybufs])
        zp = (C.c_void_p * B)(*[C.cast(b, C.c_void_p) for b in zbufs])
        yl = (C.c_size_t * B)(*[len(s) for s in ys])
        zl = (C.c_size_t * B)(*[len(s) for s in zs])
        sc = self._vbr_scales(B, **kw)
        if single:
            _lib.call("mlic_decompress_batch_stream", h, self._stream(), C.cast(ybufs[0], C.c_void_p), len(ys[0]), zp,
                      zl, B, hz, wz, x_hat.data_ptr(), sc.ctypes.data)
        else:
            _lib.call("mlic_decompress_v", h, self._stream(), yp, yl, zp, zl, B, hz, wz, x_hat.data_ptr(),
                      sc.ctypes.data)
        torch.cuda.current_stream(dev).synchronize()
        return {"x_hat": x_hat, "cost_time": time.time() - t0}

    def encoded_streams(self, b: int = 0):
        """(y_symbols, y_indexes, z_symbols) int32 arrays the coder saw for image b in the last
        compress() — the exact lists the reference hands to BufferedRansEncoder (mlicpp.py:279)."""
        ny, nz = C.c_int64(), C.c_int64()
        _lib.call("mlic_encoded_streams", self._handle, b, C.byref(ny), C.byref(nz), None, None, None)
        ys, yi, zs = np.zeros(ny.value, np.int32), np.zeros(ny.value, np.int32), np.zeros(nz.value, np.int32)
        _lib.call("mlic_encoded_streams", self._handle, b, C.byref(ny), C.byref(nz), ys.ctypes.data,
                  yi.ctypes.data, zs.ctypes.data)
        return ys, yi, zs

    def likelihood_bits(self, b: int = 0):
        """(y_bits, z_bits): sum of -log2 of image b's y / z likelihoods in the last compress(),
        computed on the device; bpp_lik = (y_bits + z_bits) / (H * W) (loss/rd_loss.py:42-45)."""
        yb, zb = C.c_double(), C.c_double()
        _lib.call("mlic_encoded_bits", self._handle, b, C.byref(yb), C.byref(zb))
        return yb.value, zb.value

    def aux_loss(self):
        """compressai EntropyBottleneck.loss(): |logits_cumulative(quantiles) - target| (training aid)."""
        eb = self.entropy_bottleneck
        p = {k: v.detach().cpu().float() for k, v in eb._parameters.items()}
        logits = entropy._logits_cumulative(p, p["quantiles"])
        return torch.abs(logits - eb._buffers["target"].detach().cpu()).sum()

    def run_module(self, which: str, idx: int, in0: torch.Tensor, in1: Optional[torch.Tensor] = None,
                   out_shape=None) -> torch.Tensor:
        """Single-module execution through the C ABI (tests/profiling)."""
        h = self._ensure_handle(in0.device)
        B, Cin, H, W = in0.shape
        out = self._out(out_shape, in0.device)
        _lib.call("mlic_run_module", h, self._stream(), which.encode(), idx, in0.contiguous().data_ptr(),
                  None if in1 is None else in1.contiguous().data_ptr(), B, Cin, H, W, out.data_ptr())
        return out


class MLICPlusPlusSD(MLICPlusPlus):
    """MLICPP_M_SMALL_DEC (models/mlicpp_small_decoder.py:16-83)."""

    def __init__(self, config=None, name: str = "MLICPP_M_SMALL_DEC", **kw):
        super().__init__(config, name=name, **kw)


class MLICPlusPlusVbr(MLICPlusPlus):
    """Variable-rate MLIC++ (models/mlicpp_vbr.py): forward(x, stage=2, s, inputscale) with the
    Gain[s] scale/rescale around the rounding (no_quantoffset = True); compress/decompress use the
    same consistent scale (the reference's VBR coder paths are broken)."""

    def __init__(self, config=None, name: str = "MLICPP_L_VBR", **kw):
        super().__init__(config, name=name, **kw)
        self.lmbda = list(spec.vbr_lambdas(name))
        self.levels = len(self.lmbda)

    def _vbr_scales(self, B: int, stage: int = 2, s=1, inputscale=0, coder: bool = False, **kw) -> np.ndarray:
        """mlicpp_vbr.py:122-137: scale = inputscale if given, else Gain[s] (clamped to the levels);
        the coder paths use |Gain[s]| (mlicpp_vbr.py:543, 899).  `s` / `inputscale` may be one value
        for the batch or one per image (BASELINE config 5)."""
        if stage != 2:
            raise ValueError("only the inference stage (stage=2) is supported")
        g = self.Gain.detach().float().cpu().numpy()
        if coder:
            g = np.abs(g)

        def per_image(v):
            a = np.asarray(v.detach().cpu() if torch.is_tensor(v) else v).reshape(-1)
            if a.size == 1:
                return np.repeat(a, B)
            if a.size != B:
                raise ValueError(f"expected 1 or {B} per-image values, got {a.size}")
            return a
        ins = per_image(inputscale).astype(np.float64)
        lv = np.clip(per_image(s).astype(np.int64), 0, len(g) - 1)
        out = np.where(ins != 0, ins, g[lv]).astype(np.float32)
        return np.ascontiguousarray(out)

    def forward(self, x, stage: int = 2, s=1, inputscale=0):
        return super().forward(x, stage=stage, s=s, inputscale=inputscale)

    def compress(self, x, stage: int = 2, s=1, inputscale=0, batch_stream: bool = False):
        return super().compress(x, batch_stream=batch_stream, stage=stage, s=s, inputscale=inputscale, coder=True)

    def decompress(self, strings, shape, stage: int = 2, s=1, inputscale=0):
        return super().decompress(strings, shape, stage=stage, s=s, inputscale=inputscale, coder=True)


class MLICPlusPlusSDVbr(MLICPlusPlusVbr):
    """MLICPP_M_SMALL_DEC_VBR (models/mlicpp_sd_vbr.py:19-1226): the small-decoder tree of
    mlicpp_small_decoder.py with mlicpp_vbr.py's stage-2 Gain[s] scale/rescale (forward / compress /
    decompress are line-for-line those of mlicpp_vbr.py), over five levels (Gain 0.002424 .. 1)."""

    def __init__(self, config=None, name: str = "MLICPP_M_SMALL_DEC_VBR", **kw):
        super().__init__(config, name=name, **kw)


def model_config(model_name: str = "MLICPP_S"):
    """config/config.py:19-62."""
    return spec.get_config(model_name)


def get_model(model_name: str) -> MLICPlusPlus:
    """models/model_loader.py:4-18 (+ MLICPP_L_VBR)."""
    cfg = spec.get_config(model_name)
    if cfg.small_decoder and cfg.vbr:
        return MLICPlusPlusSDVbr(name=model_name)
    if cfg.small_decoder:
        return MLICPlusPlusSD(name=model_name)
    if cfg.vbr:
        return MLICPlusPlusVbr(name=model_name)
    return MLICPlusPlus(name=model_name)
