"""Energy-aware step throttling (reference `opt_ops/energy/power_monitor.{h,cpp}`).

The policy and the telemetry reader are native C++ (`csrc/runtime/power_monitor.cpp`, bound as
`_C.runtime.PowerMonitor`); this module is the Python-side entry point:

* `PowerConfig` / `PowerMonitor` — the reference's battery/temperature → frequency → sleep policy
  (`power_monitor.cpp:70-112`), deterministic `"a-b:ms,c-:ms"` override schedules (`:28-68`) and
  manual readings (`:19-22`); with `use_gpu_telemetry` the inputs come from the MI355X's own power
  and junction temperature instead of mocked battery values.
* `read_gpu_telemetry(index)` — one sample of the GPU's power / temperature sensors.
* `from_args(ns)` — build a monitor from the CLIs' `--pm_*` flags (None when throttling is off).
"""
from __future__ import annotations


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


__all__ = ["PowerConfig", "PowerMonitor", "read_gpu_telemetry", "from_args"]
