"""EnergyMeter (mobilefinetuner_amd.energy): trapezoid integration of sampled GPU power, J/token,
and the no-telemetry case -- on a synthetic reader (CPU)."""
import time

from mobilefinetuner_amd.energy import EnergyMeter


def test_energy_meter_integrates_constant_power():
    m = EnergyMeter(interval=0.01, reader=lambda i: {"ok": True, "power_w": 500.0})
    with m:
        time.sleep(0.2)
    r = m.report(tokens=1000)
    assert r["ok"] and r["samples"] >= 3
    assert abs(r["mean_w"] - 500.0) < 1e-6
    assert abs(r["joules"] - 500.0 * r["seconds"]) < 1e-6
    assert abs(r["joules_per_token"] - r["joules"] / 1000) < 1e-12


def test_energy_meter_trapezoid_on_a_ramp():
    t0 = [None]

    def ramp(i):  # power rising 1000 W/s from 100 W
        now = time.monotonic()
        if t0[0] is None:
            t0[0] = now
        return {"ok": True, "power_w": 100.0 + 1000.0 * (now - t0[0])}

    m = EnergyMeter(interval=0.005, reader=ramp)
    with m:
        time.sleep(0.1)
    r = m.report()
    s = r["seconds"]
    exact = 100.0 * s + 500.0 * s * s  # integral of a linear ramp: the trapezoid rule is exact
    assert abs(r["joules"] - exact) < 0.02 * exact


def test_energy_meter_without_telemetry():
    m = EnergyMeter(interval=0.01, reader=lambda i: {"ok": False, "power_w": 0.0})
    with m:
        time.sleep(0.03)
    assert m.report(10) == {"ok": False, "reason": "no GPU power telemetry"}


def test_pci_power_reader_unknown_bus():
    from mobilefinetuner_amd.energy import pci_power_reader
    assert pci_power_reader("") is None
    assert pci_power_reader("ffff:ff:ff.7") is None
