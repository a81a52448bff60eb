"""compressai.models.CompressionModel restated (1.2.6)."""
import torch.nn as nn
from .entropy_models import EntropyBottleneck, GaussianConditional


class CompressionModel(nn.Module):
    def __init__(self, entropy_bottleneck_channels=None, init_weights=None):
        super().__init__()
        if entropy_bottleneck_channels is not None:
            self.entropy_bottleneck = EntropyBottleneck(entropy_bottleneck_channels)

    def aux_loss(self):
        return sum(m.loss() for m in self.modules() if isinstance(m, EntropyBottleneck))

    def update(self, scale_table=None, force=False):
        updated = False
        for _, m in self.named_modules():
            if isinstance(m, EntropyBottleneck):
                updated |= m.update(force=force)
        return updated
