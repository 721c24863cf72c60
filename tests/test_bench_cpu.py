"""bench.py's roofline arithmetic with a fake kernel timer (no GPU): every per-step figure
divides by the steps the timer actually recorded, not by --steps."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


class FakeTimer:
    """Records like dsgan_hip.functional.KernelTimer over `steps` identical steps: per step, 92
    pwgemm launches of 61 us each and 10 tconv launches of 70 us each."""

    def __init__(self, steps):
        self.steps = steps

    def families(self):
        s = self.steps
        return {"pwgemm_kernel": [92 * s, 92 * s * 0.061, 92 * s * 21.17e9, 92 * s * 161.95e6],
                "tconv_kernel": [10 * s, 10 * s * 0.070, 10 * s * 4e9, 10 * s * 20e6]}

    def summary(self):
        f = self.families().values()
        return dict(launches=sum(v[0] for v in f), total_ms=sum(v[1] for v in f), flops=sum(v[2] for v in f))


def _block(recorded_steps):
    t = FakeTimer(recorded_steps)
    return bench.roofline_block(t.summary(), t.families(), recorded_steps, bench.PEAK_BF16_TFLOPS, "fake")


def test_per_step_fields_use_the_recorded_steps():
    for recorded in (1, 2, 20):
        r = _block(recorded)
        assert r["timing_steps"] == recorded
        assert r["kernel"] == "pwgemm_kernel"
        assert r["launches_per_step"] == 92
        assert abs(r["kernel_ms_per_step"] - 92 * 0.061) < 1e-3
        assert r["all_contractions"]["launches_per_step"] == 102
        assert abs(r["all_contractions"]["ms_per_step"] - (92 * 0.061 + 10 * 0.070)) < 1e-3
        assert abs(r["families"]["tconv_kernel"]["ms_per_step"] - 0.70) < 1e-3
        assert r["families"]["pwgemm_kernel"]["launches_per_step"] == 92


def test_per_launch_fields_do_not_depend_on_steps():
    a, b = _block(1), _block(20)
    for k in ("frac", "achieved", "avg_launch_us", "algorithmic_bytes_per_launch", "bound"):
        assert a[k] == b[k]
    # 161.95 MB in 61 us = 2.655 TB/s: HBM-bound (its 21.17 GFLOP need 8.5 us at 2.5 PF)
    assert a["bound"] == "hbm"
    assert abs(a["achieved"] - 161.95e6 / 61e-6 / 1e9) < 1.0
    assert abs(a["avg_launch_us"] - 61.0) < 0.05


def test_pmc_traffic_feeds_waste_ratio():
    t = FakeTimer(1)
    r = bench.roofline_block(t.summary(), t.families(), 1, bench.PEAK_BF16_TFLOPS, "fake",
                             {"pwgemm_kernel": {"traffic_bytes_per_launch": 185.3e6}}, "x",
                             {"pwgemm_kernel": {"mfma_busy": 0.14}}, "y")
    assert r["traffic"] == 185.3e6
    assert abs(r["waste_ratio"] - 185.3 / 161.95) < 1e-3
    assert r["mfma"]["pmc_mfma_busy"] == 0.14
