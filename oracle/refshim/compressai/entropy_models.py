"""compressai.entropy_models restated (compressai 1.2.6 semantics).

EntropyModel.quantize/dequantize, GaussianConditional (likelihood, build_indexes,
update/CDF tables) and EntropyBottleneck (factorized prior).  The C++ helper
pmf_to_quantized_cdf (compressai/cpp_exts/ops/ops.cpp) is restated in Python in
`pmf_to_quantized_cdf` below.  Test infrastructure only.
"""
import math

import numpy as np
import scipy.stats
import torch
import torch.nn as nn
import torch.nn.functional as F

from .ops import LowerBound


def pmf_to_quantized_cdf(pmf, precision=16):
    """compressai ops.cpp pmf_to_quantized_cdf: round to `precision` bits, renormalize,
    then steal frequency so that no symbol has zero frequency."""
    pmf = [float(p) for p in pmf]
    for p in pmf:
        if p < 0 or not math.isfinite(p):
            raise ValueError("invalid pmf")
    cdf = [0] * (len(pmf) + 1)
    for i, p in enumerate(pmf):
        # std::round (half away from zero) of the float product p * (1 << precision)
        cdf[i + 1] = int(math.floor(float(np.float32(p) * np.float32(1 << precision)) + 0.5))
    total = sum(cdf)
    if total == 0:
        raise ValueError("zero pmf")
    cdf = [((1 << precision) * c) // total for c in cdf]
    for i in range(1, len(cdf)):
        cdf[i] += cdf[i - 1]
    cdf[-1] = 1 << precision
    for i in range(len(cdf) - 1):
        if cdf[i] == cdf[i + 1]:
            best_freq, best_steal = None, -1
            for j in range(len(cdf) - 1):
                freq = cdf[j + 1] - cdf[j]
                if freq > 1 and (best_freq is None or freq < best_freq):
                    best_freq, best_steal = freq, j
            assert best_steal != -1
            if best_steal < i:
                for j in range(best_steal + 1, i + 1):
                    cdf[j] -= 1
            else:
                assert best_steal > i
                for j in range(i + 1, best_steal + 1):
                    cdf[j] += 1
    return cdf


class EntropyModel(nn.Module):
    def __init__(self, likelihood_bound=1e-9, entropy_coder=None, entropy_coder_precision=16):
        super().__init__()
        self.entropy_coder_precision = int(entropy_coder_precision)
        self.use_likelihood_bound = likelihood_bound > 0
        if self.use_likelihood_bound:
            self.likelihood_lower_bound = LowerBound(likelihood_bound)
        self.register_buffer("_offset", torch.IntTensor())
        self.register_buffer("_quantized_cdf", torch.IntTensor())
        self.register_buffer("_cdf_length", torch.IntTensor())

    @property
    def offset(self):
        return self._offset

    @property
    def quantized_cdf(self):
        return self._quantized_cdf

    @property
    def cdf_length(self):
        return self._cdf_length

    def quantize(self, inputs, mode, means=None):
        if mode == "noise":
            return inputs + torch.empty_like(inputs).uniform_(-0.5, 0.5)
        outputs = inputs.clone()
        if means is not None:
            outputs -= means
        outputs = torch.round(outputs)
        if mode == "dequantize":
            if means is not None:
                outputs += means
            return outputs
        assert mode == "symbols", mode
        return outputs.int()

    def dequantize(self, inputs, means=None, dtype=torch.float):
        if means is not None:
            outputs = inputs.type_as(means)
            outputs += means
        else:
            outputs = inputs.type(dtype)
        return outputs

    def _pmf_to_cdf(self, pmf, tail_mass, pmf_length, max_length):
        cdf = torch.zeros((len(pmf_length), max_length + 2), dtype=torch.int32)
        for i, p in enumerate(pmf):
            prob = torch.cat((p[: pmf_length[i]], tail_mass[i]), dim=0)
            _cdf = pmf_to_quantized_cdf(prob.tolist(), self.entropy_coder_precision)
            cdf[i, : len(_cdf)] = torch.tensor(_cdf, dtype=torch.int32)
        return cdf


class GaussianConditional(EntropyModel):
    def __init__(self, scale_table, *args, scale_bound=0.11, tail_mass=1e-9, **kwargs):
        super().__init__(*args, **kwargs)
        self.register_buffer("scale_table", self._prepare_scale_table(scale_table) if scale_table else torch.Tensor())
        self.register_buffer("scale_bound", torch.Tensor([float(scale_bound)]) if scale_bound is not None else None)
        self.tail_mass = float(tail_mass)
        self.lower_bound_scale = LowerBound(scale_bound)

    @staticmethod
    def _prepare_scale_table(scale_table):
        return torch.Tensor(tuple(float(s) for s in scale_table))

    def _standardized_cumulative(self, inputs):
        half = float(0.5)
        const = float(-(2 ** -0.5))
        return half * torch.erfc(const * inputs)

    @staticmethod
    def _standardized_quantile(quantile):
        return scipy.stats.norm.ppf(quantile)

    def update_scale_table(self, scale_table, force=False):
        if self._offset.numel() > 0 and not force:
            return False
        self.scale_table = self._prepare_scale_table(scale_table)
        self.update()
        return True

    def update(self):
        multiplier = -self._standardized_quantile(self.tail_mass / 2)
        pmf_center = torch.ceil(self.scale_table * multiplier).int()
        pmf_length = 2 * pmf_center + 1
        max_length = torch.max(pmf_length).item()
        samples = torch.abs(torch.arange(max_length).int() - pmf_center[:, None])
        samples_scale = self.scale_table.unsqueeze(1)
        samples = samples.float()
        samples_scale = samples_scale.float()
        upper = self._standardized_cumulative((0.5 - samples) / samples_scale)
        lower = self._standardized_cumulative((-0.5 - samples) / samples_scale)
        pmf = upper - lower
        tail_mass = 2 * lower[:, :1]
        self._quantized_cdf = self._pmf_to_cdf(pmf, tail_mass, pmf_length, max_length)
        self._offset = -pmf_center
        self._cdf_length = pmf_length + 2

    def _likelihood(self, inputs, scales, means=None):
        half = float(0.5)
        values = inputs - means if means is not None else inputs
        scales = self.lower_bound_scale(scales)
        values = torch.abs(values)
        upper = self._standardized_cumulative((half - values) / scales)
        lower = self._standardized_cumulative((-half - values) / scales)
        return upper - lower

    def forward(self, inputs, scales, means=None, training=None):
        if training is None:
            training = self.training
        outputs = self.quantize(inputs, "noise" if training else "dequantize", means)
        likelihood = self._likelihood(outputs, scales, means)
        if self.use_likelihood_bound:
            likelihood = self.likelihood_lower_bound(likelihood)
        return outputs, likelihood

    def build_indexes(self, scales):
        scales = self.lower_bound_scale(scales)
        indexes = scales.new_full(scales.size(), len(self.scale_table) - 1).int()
        for s in self.scale_table[:-1]:
            indexes -= (scales <= s).int()
        return indexes


class EntropyBottleneck(EntropyModel):
    def __init__(self, channels, *args, tail_mass=1e-9, init_scale=10, filters=(3, 3, 3, 3), **kwargs):
        super().__init__(*args, **kwargs)
        self.channels = int(channels)
        self.filters = tuple(int(f) for f in filters)
        self.init_scale = float(init_scale)
        self.tail_mass = float(tail_mass)
        filters = (1,) + self.filters + (1,)
        scale = self.init_scale ** (1 / (len(self.filters) + 1))
        for i in range(len(self.filters) + 1):
            init = np.log(np.expm1(1 / scale / filters[i + 1]))
            matrix = torch.Tensor(channels, filters[i + 1], filters[i])
            matrix.data.fill_(init)
            self.register_parameter(f"_matrix{i:d}", nn.Parameter(matrix))
            bias = torch.Tensor(channels, filters[i + 1], 1)
            nn.init.uniform_(bias, -0.5, 0.5)
            self.register_parameter(f"_bias{i:d}", nn.Parameter(bias))
            if i < len(self.filters):
                factor = torch.Tensor(channels, filters[i + 1], 1)
                nn.init.zeros_(factor)
                self.register_parameter(f"_factor{i:d}", nn.Parameter(factor))
        self.quantiles = nn.Parameter(torch.Tensor(channels, 1, 3))
        init = torch.Tensor([-self.init_scale, 0, self.init_scale])
        self.quantiles.data = init.repeat(self.quantiles.size(0), 1, 1)
        target = np.log(2 / self.tail_mass - 1)
        self.register_buffer("target", torch.Tensor([-target, 0, target]))

    def _get_medians(self):
        return self.quantiles[:, :, 1:2]

    def _logits_cumulative(self, inputs, stop_gradient):
        logits = inputs
        for i in range(len(self.filters) + 1):
            matrix = getattr(self, f"_matrix{i:d}")
            logits = torch.matmul(F.softplus(matrix), logits)
            logits += getattr(self, f"_bias{i:d}")
            if i < len(self.filters):
                logits += torch.tanh(getattr(self, f"_factor{i:d}")) * torch.tanh(logits)
        return logits

    def _likelihood(self, inputs):
        # compressai 1.2.x: plain sigmoid difference.  PARITY UNPINNED: compressai is not installed here
        # and nothing in the reference tree holds its output; the form restated is 1.2.6's
        # EntropyBottleneck._likelihood as published -- lower = self._logits_cumulative(inputs - half),
        # upper = self._logits_cumulative(inputs + half), likelihood = sigmoid(upper) - sigmoid(lower)
        # (1.1.x instead took sign = -sign(lower + upper) and abs(sigmoid(sign * upper) - sigmoid(sign *
        # lower))); update() builds the pmf from the same expression with stop_gradient=True
        half = float(0.5)
        lower = self._logits_cumulative(inputs - half, stop_gradient=False)
        upper = self._logits_cumulative(inputs + half, stop_gradient=False)
        return torch.sigmoid(upper) - torch.sigmoid(lower)

    def update(self, force=False):
        if self._offset.numel() > 0 and not force:
            return False
        medians = self.quantiles[:, 0, 1]
        minima = torch.clamp(torch.ceil(medians - self.quantiles[:, 0, 0]).int(), min=0)
        maxima = torch.clamp(torch.ceil(self.quantiles[:, 0, 2] - medians).int(), min=0)
        self._offset = -minima
        pmf_start = medians - minima
        pmf_length = maxima + minima + 1
        max_length = pmf_length.max().item()
        samples = torch.arange(max_length)
        samples = samples[None, :] + pmf_start[:, None, None]
        half = float(0.5)
        with torch.no_grad():
            # compressai 1.2.x: pmf, lower, upper = self._likelihood(samples, stop_gradient=True),
            # i.e. the plain sigmoid difference (1.1.x used the sign trick with abs)
            lower = self._logits_cumulative(samples - half, stop_gradient=True)
            upper = self._logits_cumulative(samples + half, stop_gradient=True)
            pmf = torch.sigmoid(upper) - torch.sigmoid(lower)
            pmf = pmf[:, 0, :]
            tail_mass = torch.sigmoid(lower[:, 0, :1]) + torch.sigmoid(-upper[:, 0, -1:])
        self._quantized_cdf = self._pmf_to_cdf(pmf, tail_mass, pmf_length, max_length)
        self._cdf_length = pmf_length + 2
        return True

    def forward(self, x, training=None):
        if training is None:
            training = self.training
        perm = np.arange(len(x.shape))
        perm[0], perm[1] = perm[1], perm[0]
        inv_perm = np.arange(len(x.shape))[np.argsort(perm)]
        x = x.permute(*perm).contiguous()
        shape = x.size()
        values = x.reshape(x.size(0), 1, -1)
        outputs = self.quantize(values, "noise" if training else "dequantize", self._get_medians())
        likelihood = self._likelihood(outputs)
        if self.use_likelihood_bound:
            likelihood = self.likelihood_lower_bound(likelihood)
        outputs = outputs.reshape(shape).permute(*inv_perm).contiguous()
        likelihood = likelihood.reshape(shape).permute(*inv_perm).contiguous()
        return outputs, likelihood

    @staticmethod
    def _build_indexes(size):
        dims = len(size)
        view_dims = np.ones((dims,), dtype=np.int64)
        view_dims[1] = -1
        indexes = torch.arange(size[1]).view(*view_dims).int()
        return indexes.repeat(size[0], 1, *size[2:])

    def compress_symbols(self, x):
        """(symbols, indexes) that EntropyModel.compress would hand to the coder."""
        indexes = self._build_indexes(x.size())
        medians = self._get_medians().detach().reshape(1, -1, 1, 1).expand(x.size(0), -1, 1, 1)
        return self.quantize(x, "symbols", medians), indexes


class EntropyBottleneckVbr(EntropyBottleneck):  # imported by mlicpp_vbr.py; unused with vr_entbttlnck=None
    pass


def _eb_compress(self, x):
    """EntropyBottleneck.compress stand-in: the 'string' carries the int symbols
    round(z - median) (the rANS bytes themselves are produced by mlic_amd's coder)."""
    med = self._get_medians().detach().reshape(1, -1, 1, 1)
    sym = torch.round(x - med).int()
    return [("zsym", sym[i].clone()) for i in range(sym.shape[0])]


def _eb_decompress(self, strings, size):
    med = self._get_medians().detach().reshape(1, -1, 1, 1)
    sym = torch.stack([s[1] for s in strings]).reshape(len(strings), -1, *size)
    return sym.float() + med


EntropyBottleneck.compress = _eb_compress
EntropyBottleneck.decompress = _eb_decompress
