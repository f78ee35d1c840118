"""Energy-aware step throttling (reference `opt_ops/energy/power_monitor.{h,cpp}`).

The policy and the telemetry reader are native C++ (`csrc/runtime/power_monitor.cpp`, bound as
`_C.runtime.PowerMonitor`); this module is the Python-side entry point:

* `PowerConfig` / `PowerMonitor` — the reference's battery/temperature → frequency → sleep policy
  (`power_monitor.cpp:70-112`), deterministic `"a-b:ms,c-:ms"` override schedules (`:28-68`) and
  manual readings (`:19-22`); with `use_gpu_telemetry` the inputs come from the MI355X's own power
  and junction temperature instead of mocked battery values.
* `read_gpu_telemetry(index)` — one sample of the GPU's power / temperature sensors.
* `from_args(ns)` — build a monitor from the CLIs' `--pm_*` flags (None when throttling is off).
* `EnergyMeter` — integrates the GPU's socket power over a run on a sampling thread (trapezoid rule over
  the timestamped samples) and reports joules, mean / peak power and joules per token: the energy side of
  the reference's energy-aware training, measured on the accelerator rather than a phone battery.
"""
from __future__ import annotations

import threading
import time


def _rt():
    from .._ext import native
    return native().runtime


def PowerConfig():  # noqa: N802 - mirrors the native class name
    return _rt().PowerConfig()


def PowerMonitor(cfg):  # noqa: N802
    return _rt().PowerMonitor(cfg)


def read_gpu_telemetry(index: int = 0):
    return _rt().read_gpu_telemetry(index)


def from_args(ns):
    from ..cli.common import build_power_monitor
    return build_power_monitor(ns)


def pci_power_reader(pci_bus_id: str):
    """A telemetry reader (index ignored) for the amdgpu card at `pci_bus_id` ("0000:05:00.0"), or None
    when sysfs has no such card: the card numbering of /sys/class/drm need not follow the devices a
    process sees, so the engine reports the PCI address of the GPU it runs on."""
    import glob
    import os
    want = pci_bus_id.strip().lower()
    if not want:
        return None
    for card in sorted(glob.glob("/sys/class/drm/card*/device")):
        try:
            if not os.path.realpath(card).lower().endswith(want):
                continue
        except OSError:
            continue
        hw = sorted(glob.glob(os.path.join(card, "hwmon", "hwmon*")))
        if not hw:
            return None
        files = [os.path.join(hw[0], f) for f in ("power1_average", "power1_input")]

        def read(_index=0, files=files):
            for f in files:
                try:
                    with open(f) as fh:
                        return {"ok": True, "power_w": int(fh.read().strip()) / 1e6}
                except (OSError, ValueError):
                    continue
            return {"ok": False, "power_w": 0.0}

        return read
    return None


class EnergyMeter:
    """`with EnergyMeter(gpu=0) as m: ...train...; m.report(tokens)` -> joules, mean/peak watts, J/token.

    Power is sampled every `interval` seconds on a daemon thread; the energy is the trapezoid integral
    of the (time, watts) samples, the first one taken at `__enter__` and the last at `__exit__`.
    `reader` (index -> dict with "ok" and "power_w") defaults to the native hwmon reader; tests pass a
    synthetic one.  When the sensors are unavailable (`ok` false) `report()` says so instead of
    returning a number."""

    def __init__(self, gpu: int = 0, interval: float = 0.05, reader=None):
        self.gpu, self.interval = gpu, interval
        self._read = reader or read_gpu_telemetry
        self.samples: list[tuple[float, float]] = []
        self.ok = True
        self._stop = threading.Event()
        self._thr = None

    def _sample(self):
        t = self._read(self.gpu)
        if not t.get("ok", False):
            self.ok = False
            return
        self.samples.append((time.monotonic(), float(t["power_w"])))

    def _loop(self):
        while not self._stop.wait(self.interval):
            self._sample()

    def __enter__(self):
        self.samples.clear()
        self.ok = True
        self._stop.clear()
        self._sample()
        self._thr = threading.Thread(target=self._loop, daemon=True)
        self._thr.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        self._thr.join()
        self._sample()
        return False

    def joules(self) -> float:
        s = self.samples
        return sum(0.5 * (s[i][1] + s[i - 1][1]) * (s[i][0] - s[i - 1][0]) for i in range(1, len(s)))

    def report(self, tokens: int = 0) -> dict:
        if not self.ok or len(self.samples) < 2:
            return {"ok": False, "reason": "no GPU power telemetry"}
        secs = self.samples[-1][0] - self.samples[0][0]
        j = self.joules()
        r = {"ok": True, "seconds": secs, "joules": j, "mean_w": j / secs if secs > 0 else 0.0,
             "peak_w": max(w for _, w in self.samples), "samples": len(self.samples)}
        if tokens:
            r["joules_per_token"] = j / tokens
        return r


__all__ = ["PowerConfig", "PowerMonitor", "read_gpu_telemetry", "from_args", "EnergyMeter", "pci_power_reader"]
