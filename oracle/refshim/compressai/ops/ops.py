"""compressai.ops restated: quantize_ste, LowerBound (compressai 1.2.6)."""
import torch
import torch.nn as nn


def quantize_ste(x):
    # forward value round(x) (half-to-even); straight-through gradient
    return (torch.round(x) - x).detach() + x


class LowerBound(nn.Module):
    def __init__(self, bound):
        super().__init__()
        self.register_buffer("bound", torch.Tensor([float(bound)]))

    def forward(self, x):
        return torch.max(x, self.bound)
