from .ops import quantize_ste, LowerBound  # noqa: F401
