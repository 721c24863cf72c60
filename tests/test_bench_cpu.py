"""bench.py's roofline arithmetic with a fake kernel timer (no GPU): every per-step figure
divides by the steps the timer actually recorded, not by --steps."""
import os
import sys

import pytest

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


def test_kernel_only_timing_replaces_the_bracket():
    """The dominant pointwise family's per-launch time comes from the library's kernel-only events
    (dsgan_ktimer: the GEMM kernel alone, no split-K finishing pass) when they cover the same
    launches; the C-ABI bracket stays beside it."""
    t = FakeTimer(2)
    pw_ms = [0.0593] * (92 * 2)          # the kernel alone: 59.3 us against the 61-us bracket
    r = bench.roofline_block(t.summary(), t.families(), 2, bench.PEAK_BF16_TFLOPS, "fake", pw_ms=pw_ms)
    assert abs(r["avg_launch_us"] - 59.3) < 0.05 and abs(r["bracket_avg_launch_us"] - 61.0) < 0.05
    assert r["avg_launch_timing"].startswith("kernel-only")
    assert abs(r["achieved"] - 161.95e6 / 59.3e-6 / 1e9) < 1.0
    assert abs(r["kernel_ms_per_step"] - 92 * 0.0593) < 1e-3
    # a pair count that does not match the family's calls, or unreadable pairs: the bracket
    for bad in (pw_ms[:-1], None, []):
        r = bench.roofline_block(t.summary(), t.families(), 2, bench.PEAK_BF16_TFLOPS, "fake", pw_ms=bad)
        assert abs(r["avg_launch_us"] - 61.0) < 0.05 and r["avg_launch_timing"].startswith("HIP events around")


def test_rocprof_family_average(tmp_path):
    p = tmp_path / "s.csv"
    p.write_text('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs"\n'
                 '"_ZN3dsg13pwgemm_kernelIDF16bLi2EEEvNS_6PwArgsE",30,1800000,60000.0,1.0,1,1\n'
                 '"void dsg::pwgemm_kernel<bool _Accum, int>(dsg::PwArgs)",10,580000,58000.0,1.0,1,1\n'
                 '"dsg::split_canon_kernel(dsg::RSegs)",5,50000,10000.0,1.0,1,1\n')
    avg, calls = bench.rocprof_family_avg_us(str(p), "pwgemm_kernel")
    assert calls == 40 and abs(avg - 59.5) < 1e-6


@pytest.mark.parametrize("tag", ["a", "final"])
def test_committed_bench_line_agrees_with_its_rocprof_summary(tag):
    """the committed round-6 bench line's avg_launch_us for the dominant family
    (kernel-only events) is within 5 % of the average of the same family in the committed rocprofv3
    summary of the bench command on the same tree (profiles/r06: bench_<tag>.log with rocprof_stats_<tag>.csv;
    "final" = the round's last tree)."""
    import json
    d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "r06")
    with open(os.path.join(d, "bench_%s.log" % tag)) as f:
        line = json.loads([x for x in f if x.startswith("{")][-1])
    r = line["roofline"]
    assert r["avg_launch_timing"].startswith("kernel-only")
    avg, calls = bench.rocprof_family_avg_us(os.path.join(d, "rocprof_stats_%s.csv" % tag), r["kernel"])
    assert calls > 0
    assert abs(r["avg_launch_us"] - avg) <= 0.05 * avg, (r["avg_launch_us"], avg)
