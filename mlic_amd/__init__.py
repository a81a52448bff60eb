"""mlic_amd: MI355X-native (gfx950) MLIC++ encode/decode behind the CompressAI-style API.

    from mlic_amd import get_model
    net = get_model("MLICPP_L").cuda().eval()
"""
from .models import MLICPlusPlus, MLICPlusPlusSD, MLICPlusPlusSDVbr, MLICPlusPlusVbr, get_model, model_config  # noqa: F401
from .spec import CONFIGS  # noqa: F401

__all__ = ["MLICPlusPlus", "MLICPlusPlusSD", "MLICPlusPlusSDVbr", "MLICPlusPlusVbr", "get_model", "model_config", "CONFIGS"]
