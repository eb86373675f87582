"""Device description (CU count, clock) through the native library."""
from __future__ import annotations

from .. import _native


def info(dev: int = 0) -> dict:
    lib = _native.require_gpu_lib()
    return {
        "device": dev,
        "count": lib.otc_device_count(),
        "cus": lib.otc_device_cus(dev),
        "clock_hz": lib.otc_device_clock_khz(dev) * 1e3,
        "build": lib.otc_build_info().decode(),
    }
