"""Entropy-model tables and the standalone rANS coder (compressai replacement, host side).

GaussianConditional.update() / EntropyBottleneck.update() of compressai 1.2.6 compute a pmf per
table with a few torch CPU ops and quantize it with the C++ `pmf_to_quantized_cdf`; this module
does the same (torch CPU for the pmf = glue, libmlic_hip for the quantisation), so the resulting
`_quantized_cdf` / `_cdf_length` / `_offset` buffers — and therefore the bitstreams — match the
reference's (mlicpp.py:470-475; utils/func.py:16-19).
"""
from __future__ import annotations

import ctypes as C
import math
from typing import Tuple

import numpy as np
import scipy.stats
import torch
import torch.nn.functional as F

from . import _lib

PRECISION = 16


def get_scale_table(min: float = 0.11, max: float = 256, levels: int = 64) -> torch.Tensor:  # noqa: A002
    """utils/func.py:16-19."""
    return torch.exp(torch.linspace(math.log(min), math.log(max), levels))


def pmf_to_quantized_cdf(pmf: np.ndarray, precision: int = PRECISION) -> np.ndarray:
    pmf = np.ascontiguousarray(pmf, dtype=np.float32)
    out = np.zeros(pmf.size + 1, np.int32)
    _lib.call("mlic_pmf_to_quantized_cdf", pmf.ctypes.data, int(pmf.size), int(precision), out.ctypes.data)
    return out


def _pmf_to_cdf(pmf: torch.Tensor, tail_mass: torch.Tensor, pmf_length: torch.Tensor, max_length: int):
    cdf = torch.zeros((len(pmf_length), max_length + 2), dtype=torch.int32)
    for i, p in enumerate(pmf):
        prob = torch.cat((p[: pmf_length[i]], tail_mass[i]), dim=0)
        q = pmf_to_quantized_cdf(prob.numpy())
        cdf[i, : q.size] = torch.from_numpy(q)
    return cdf


def _std_cumulative(x: torch.Tensor) -> torch.Tensor:
    return 0.5 * torch.erfc(float(-(2 ** -0.5)) * x)


def gaussian_tables(scale_table: torch.Tensor, tail_mass: float = 1e-9):
    """compressai GaussianConditional.update(): (quantized_cdf, cdf_length, offset)."""
    scale_table = torch.Tensor(tuple(float(s) for s in scale_table))
    multiplier = -scipy.stats.norm.ppf(tail_mass / 2)
    pmf_center = torch.ceil(scale_table * multiplier).int()
    pmf_length = 2 * pmf_center + 1
    max_length = int(torch.max(pmf_length).item())
    samples = torch.abs(torch.arange(max_length).int() - pmf_center[:, None]).float()
    samples_scale = scale_table.unsqueeze(1).float()
    upper = _std_cumulative((0.5 - samples) / samples_scale)
    lower = _std_cumulative((-0.5 - samples) / samples_scale)
    pmf = upper - lower
    tail = 2 * lower[:, :1]
    cdf = _pmf_to_cdf(pmf, tail, pmf_length, max_length)
    return cdf, (pmf_length + 2).int(), (-pmf_center).int(), scale_table


def _logits_cumulative(params, x):
    logits = x
    for i in range(5):
        logits = torch.matmul(F.softplus(params[f"_matrix{i}"]), logits)
        logits = logits + params[f"_bias{i}"]
        if i < 4:
            logits = logits + torch.tanh(params[f"_factor{i}"]) * torch.tanh(logits)
    return logits


def bottleneck_pmf(params: dict, sign_trick: bool = False):
    """The per-channel pmf, tail mass, pmf lengths and offsets EntropyBottleneck.update() quantises.

    compressai >= 1.2 (the reference pins 1.2.6, requirements.txt:31) takes the pmf from
    `_likelihood(samples)`, i.e. the plain `sigmoid(upper) - sigmoid(lower)`.  `sign_trick=True` gives
    the 1.1-era `abs(sigmoid(s*upper) - sigmoid(s*lower))`, s = -sign(lower + upper), kept only so a
    test can count the quantised-CDF entries the two forms disagree on."""
    q = params["quantiles"].detach().cpu().float()
    p = {k: v.detach().cpu().float() for k, v in params.items()}
    medians = q[:, 0, 1]
    minima = torch.clamp(torch.ceil(medians - q[:, 0, 0]).int(), min=0)
    maxima = torch.clamp(torch.ceil(q[:, 0, 2] - medians).int(), min=0)
    offset = -minima
    pmf_start = medians - minima
    pmf_length = maxima + minima + 1
    max_length = int(pmf_length.max().item())
    samples = torch.arange(max_length)[None, :] + pmf_start[:, None, None]
    lower = _logits_cumulative(p, samples - 0.5)
    upper = _logits_cumulative(p, samples + 0.5)
    if sign_trick:
        sign = -torch.sign(lower + upper)
        pmf = torch.abs(torch.sigmoid(sign * upper) - torch.sigmoid(sign * lower))
    else:
        pmf = torch.sigmoid(upper) - torch.sigmoid(lower)
    pmf = pmf[:, 0, :]
    tail = torch.sigmoid(lower[:, 0, :1]) + torch.sigmoid(-upper[:, 0, -1:])
    return pmf, tail, pmf_length, max_length, offset


@torch.no_grad()
def bottleneck_tables(params: dict, sign_trick: bool = False):
    """compressai 1.2.6 EntropyBottleneck.update(): (quantized_cdf, cdf_length, offset)."""
    pmf, tail, pmf_length, max_length, offset = bottleneck_pmf(params, sign_trick)
    cdf = _pmf_to_cdf(pmf, tail, pmf_length, max_length)
    return cdf, (pmf_length + 2).int(), offset.int()


def _tab_args(cdf, length, offset):
    cdf = np.ascontiguousarray(cdf.numpy() if torch.is_tensor(cdf) else cdf, dtype=np.int32)
    length = np.ascontiguousarray(np.asarray(length).reshape(-1), dtype=np.int32)
    offset = np.ascontiguousarray(np.asarray(offset).reshape(-1), dtype=np.int32)
    return cdf, length, offset


def rans_encode(symbols, indexes, cdf, length, offset) -> bytes:
    """compressai RansEncoder.encode_with_indexes (byte-compatible)."""
    s = np.ascontiguousarray(np.asarray(symbols).reshape(-1), dtype=np.int32)
    ix = np.ascontiguousarray(np.asarray(indexes).reshape(-1), dtype=np.int32)
    cdf, length, offset = _tab_args(cdf, length, offset)
    cap = 4 * (2 * s.size + 16) + 64
    buf = C.create_string_buffer(cap)
    written = C.c_size_t(0)
    _lib.call("mlic_rans_encode", s.ctypes.data, ix.ctypes.data, s.size, cdf.ctypes.data, length.ctypes.data,
              offset.ctypes.data, cdf.shape[0], cdf.shape[1], buf, cap, C.byref(written))
    return C.string_at(buf, written.value)


def rans_decode(data: bytes, indexes, cdf, length, offset) -> np.ndarray:
    """compressai RansDecoder.decode_with_indexes."""
    ix = np.ascontiguousarray(np.asarray(indexes).reshape(-1), dtype=np.int32)
    cdf, length, offset = _tab_args(cdf, length, offset)
    out = np.zeros(ix.size, np.int32)
    _lib.call("mlic_rans_decode", data, len(data), ix.ctypes.data, ix.size, cdf.ctypes.data, length.ctypes.data,
              offset.ctypes.data, cdf.shape[0], cdf.shape[1], out.ctypes.data)
    return out
