"""Socket energy, power, clock and power-limit residency of one GPU over a
time window, read in process through the ``amdsmi`` library.

Every AES kernel on MI355X runs against the package power limit (PPT): at the
cap, throughput follows energy per byte, and a box that holds a lower clock
reads as "slower" unless the record carries the power side too (docs/PERF.md).
``PowerMeter`` brackets a timed region:

* ``joules``     -- socket energy counter delta (``amdsmi_get_energy_count``,
  counter x resolution), so ``avg_socket_w`` = joules / window is an average
  over the whole window, not a sampled guess;
* ``ppt_residency`` -- fraction of the window the PPT limit was active
  (``ppt_residency_acc`` / ``accumulation_counter`` deltas of the GPU metrics
  table, the counters ``amd-smi metric -v`` prints as PPT_ACCUMULATED);
* ``gfxclk_mhz_mean`` / min / max -- the 8 XCDs' current GFX clocks, sampled
  every ``sample_s`` by a background thread (with the socket power samples);
* ``xgmi_read_kb`` / ``xgmi_write_kb`` -- deltas of the xGMI data counters
  (summed over links; the metrics table counts KB), i.e. the traffic this GPU
  really moved over xGMI in the window.

The reference's only metric is wall-clock microseconds
(/root/reference/test.c:31-40); this is the MI355X-specific addition the
power cap makes necessary.  Nothing here touches HIP: the meter can be created
before or after the GPU is initialised (it never forks or execs).
"""
from __future__ import annotations

import threading
import time


def _bdf_of_torch_device(index: int) -> str | None:
    try:
        import torch

        p = torch.cuda.get_device_properties(index)
        return "%04x:%02x:%02x" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
    except Exception:
        return None


class PowerMeter:
    """``m = PowerMeter(hip_index); m.start(); ...; stats = m.stop()``.

    ``stats["available"]`` is False (with ``reason``) when amdsmi cannot read
    this GPU -- no driver in the container, permissions -- and the caller
    reports that instead of numbers."""

    def __init__(self, hip_index: int = 0, sample_s: float = 0.05, torch_bdf: bool = True):
        """torch_bdf: find the GPU by the PCI address torch reports for HIP
        device ``hip_index`` (imports torch and initialises HIP: seconds in a
        fresh process); False: the amdsmi handle of the same index (right when
        no device is hidden from HIP, e.g. a watcher process beside a
        benchmark that owns the GPU)."""
        self.hip_index = hip_index
        self.sample_s = sample_s
        self.reason = ""
        self.prime_s = None
        self._h = None
        self._smi = None
        try:
            import amdsmi

            amdsmi.amdsmi_init()
            self._smi = amdsmi
            handles = amdsmi.amdsmi_get_processor_handles()
            want = _bdf_of_torch_device(hip_index) if torch_bdf else None
            if want is not None:
                for h in handles:
                    if amdsmi.amdsmi_get_gpu_device_bdf(h).lower().startswith(want):
                        self._h = h
                        break
            if self._h is None and hip_index < len(handles):
                self._h = handles[hip_index]  # same enumeration order as HIP when nothing is hidden
            if self._h is None:
                self.reason = f"no amdsmi handle for HIP device {hip_index} (bdf {want})"
            else:
                # the first metrics / energy read of a process takes ~1.3 s on
                # the box: pay it here, not inside start() (which would open
                # the window that much after the caller's timed region began)
                t0 = time.perf_counter()
                self._metrics()
                self._energy_j()
                self.prime_s = time.perf_counter() - t0
        except Exception as e:  # no driver here, or no permission on the box
            self.reason = f"amdsmi unavailable: {type(e).__name__}: {e}"
        self._samples: list[tuple[float, float, float]] = []
        self._stop = threading.Event()
        self._thr = None
        self._t0 = self._e0 = self._m0 = None
        self.start_call_s = 0.0

    @property
    def available(self) -> bool:
        return self._h is not None

    def _energy_j(self) -> float:
        r = self._smi.amdsmi_get_energy_count(self._h)
        return float(r["energy_accumulator"]) * float(r["counter_resolution"]) * 1e-6

    def _metrics(self) -> dict:
        return self._smi.amdsmi_get_gpu_metrics_info(self._h)

    def _sample(self):
        while not self._stop.is_set():
            try:
                m = self._metrics()
                clks = [c for c in m.get("current_gfxclks") or [] if isinstance(c, (int, float)) and 0 < c < 10000]
                w = m.get("current_socket_power")
                self._samples.append((time.perf_counter(), float(w) if isinstance(w, (int, float)) else float("nan"),
                                      sum(clks) / len(clks) if clks else float("nan")))
            except Exception:
                pass
            self._stop.wait(self.sample_s)

    def start(self):
        if not self.available:
            return self
        self._samples = []
        self._stop.clear()
        tc = time.perf_counter()
        self._m0 = self._metrics()
        self._e0 = self._energy_j()
        self._t0 = time.perf_counter()
        self.start_call_s = self._t0 - tc
        self._thr = threading.Thread(target=self._sample, daemon=True)
        self._thr.start()
        return self

    def stop(self, nbytes: int | None = None) -> dict:
        """Stats of the window since ``start``; with ``nbytes`` (bytes this
        GPU processed in the window) also ``joules_per_gb``."""
        if not self.available:
            return {"available": False, "reason": self.reason}
        t1 = time.perf_counter()
        e1 = self._energy_j()
        m1 = self._metrics()
        self._stop.set()
        if self._thr is not None:
            self._thr.join(timeout=2.0)
        dt = t1 - self._t0
        joules = e1 - self._e0
        out = {"available": True, "window_s": round(dt, 4), "start_call_s": round(self.start_call_s, 4),
               "joules": round(joules, 3),
               "avg_socket_w": round(joules / dt, 1) if dt > 0 else None}

        def delta(k):
            a, b = self._m0.get(k), m1.get(k)
            return b - a if isinstance(a, int) and isinstance(b, int) else None

        acc, ppt = delta("accumulation_counter"), delta("ppt_residency_acc")
        out["ppt_residency"] = round(ppt / acc, 4) if acc and ppt is not None else None
        thm = delta("socket_thm_residency_acc")
        out["socket_thermal_residency"] = round(thm / acc, 4) if acc and thm is not None else None
        for name, k in (("xgmi_read_kb", "xgmi_read_data_acc"), ("xgmi_write_kb", "xgmi_write_data_acc")):
            a, b = self._m0.get(k), m1.get(k)
            if isinstance(a, list) and isinstance(b, list):
                ds = [y - x for x, y in zip(a, b) if isinstance(x, int) and isinstance(y, int)]
                out[name] = sum(ds) if ds else None
        ws = [w for (_, w, _) in self._samples if w == w]
        cs = [c for (_, _, c) in self._samples if c == c]
        out["power_samples"] = len(ws)
        if ws:
            out["socket_w_min"], out["socket_w_max"] = min(ws), max(ws)
        if cs:
            out["gfxclk_mhz_mean"] = round(sum(cs) / len(cs), 1)
            out["gfxclk_mhz_min"], out["gfxclk_mhz_max"] = round(min(cs), 1), round(max(cs), 1)
        if nbytes:
            out["joules_per_gb"] = round(joules / (nbytes / 1e9), 4)
        return out

    def close(self):
        self._stop.set()
        if self._smi is not None:
            try:
                self._smi.amdsmi_shut_down()
            except Exception:
                pass
            self._smi = None
