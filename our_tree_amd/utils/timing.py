"""Timing helpers: hipEvent (torch.cuda.Event on ROCm) kernel timing and
wall-clock regions.  The reference only had gettimeofday around thread
spawn/join or around allocation+copies (test.c:31-40, main_ecb_e.cu:37-44)."""
from __future__ import annotations

import time
from contextlib import contextmanager


class DeviceTimer:
    """Accumulates device time between start()/stop() pairs on the current stream."""

    def __init__(self):
        import torch

        self._torch = torch
        self._pairs = []

    def start(self):
        e = self._torch.cuda.Event(enable_timing=True)
        e.record()
        self._pairs.append([e, None])

    def stop(self):
        e = self._torch.cuda.Event(enable_timing=True)
        e.record()
        self._pairs[-1][1] = e

    def elapsed_ms(self) -> float:
        self._torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in self._pairs if b is not None)


@contextmanager
def wall(result: dict, key: str = "ms"):
    t0 = time.perf_counter()
    yield
    result[key] = (time.perf_counter() - t0) * 1e3


def gbps(nbytes: int, ms: float) -> float:
    return nbytes / (ms * 1e6) if ms > 0 else float("nan")


def cycles_per_byte_per_cu(nbytes: int, ms: float, cus: int, clock_hz: float) -> float:
    """(CUs x clock x time) / bytes: the per-CU cost metric of BASELINE.json."""
    return (ms * 1e-3) * clock_hz * cus / nbytes if nbytes else float("nan")
