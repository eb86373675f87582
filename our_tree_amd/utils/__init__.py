"""Utilities: result-log formats, timing, device info."""
from . import results, timing

__all__ = ["results", "timing"]
