"""bench.py's bookkeeping (CPU): the PMC traffic record is used only for the kernels it measured
(its kernel-source hash) and the workload shape it measured; the per-class table scales the
record's per-dispatch bytes and FLOPs by dispatches per call, and reports null where the record's
dispatch count per step is not the profiled one (poly2_int's 4-dispatch calls)."""
import ctypes as C
import json
import sys
from types import SimpleNamespace

import pytest

from conftest import ROOT

sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def _args(**kw):
    a = SimpleNamespace(log_n=16, max_level=30, special_primes=10, digit_primes=12, scale_bits=40,
                        batch=32, layout="sliced")
    a.__dict__.update(kw)
    return a


def test_csrc_hash_gates_the_pmc_record(tmp_path, monkeypatch):
    rec = {"csrc_sha16": bench.csrc_sha16(), "workload": {"log_n": 16, "max_level": 30, "special_primes": 10,
                                                          "digit_primes": 12, "batch": 32, "layout": "sliced"},
           "ntt_family": {"hbm_bytes_per_launch": 1.0}, "per_kernel": {}}
    f = tmp_path / "round_traffic.json"
    monkeypatch.setattr(bench, "PMC_FILE", f)
    f.write_text(json.dumps(rec))
    assert bench.pmc_record(_args()) is not None
    assert bench.pmc_record(_args(batch=16)) is None          # another workload shape
    rec["csrc_sha16"] = "0" * 16
    f.write_text(json.dumps(rec))
    assert bench.pmc_record(_args()) is None                  # measured on other kernels
    assert bench.pmc_record() is None


def test_committed_pmc_record_is_the_trees_own():
    """The PMC record bench.py reads (profiles/rNN/pmc/round_traffic.json) measured exactly these
    kernel sources and the default workload: a kernel edit without a retaken record would leave
    the driver's line without `traffic` (tools/gpu_r06_pmc.sh + tools/pmc_traffic.py retake it)."""
    rec = bench.pmc_record(_args())
    assert rec is not None, f"{bench.PMC_FILE} was not measured on this tree's kernel sources"
    per = rec["per_kernel"]
    for cls in ("ks_rows_fin.prod", "modup_cols", "moddown_cols", "poly2_int"):
        assert per[cls]["hbm_bytes_per_launch"] > 0


class _FakeEngine:
    """engine_profile_kernels of two classes over 2 profiled steps: 'a' one dispatch per call,
    'b' three dispatches per call (as poly2_int's)."""

    def __init__(self, raw):
        self.js = json.dumps(raw).encode()
        self._h = None
        self._lib = SimpleNamespace(engine_profile_kernels=self._prof)

    def _check(self, rc):
        assert rc == 0

    def _prof(self, h, buf, cap, need):
        need._obj.value = len(self.js) + 1
        if buf is not None:
            C.memmove(buf, self.js, len(self.js))
        return 0


def test_kernel_table_scales_by_dispatches():
    raw = {"a": [20, 2.0, 20 * 1e6, 20], "b": [8, 16.0, 8 * 4e7, 24]}  # calls, ms, bytes, dispatches
    pmc = {"per_kernel": {"a": {"launches": 10, "hbm_bytes_per_launch": 2e6, "f64_flops_per_launch": 1e9},
                          "b": {"launches": 12, "hbm_bytes_per_launch": 1.4e7, "f64_flops_per_launch": 3e11}}}
    t = bench.kernel_table(_FakeEngine(raw), pmc, 2)
    assert t["a"]["dispatches_per_step"] == 10 and t["a"]["hbm_bytes_per_launch"] == 2e6
    b = t["b"]
    assert b["launches_per_step"] == 4 and b["dispatches_per_step"] == 12
    assert b["hbm_bytes_per_launch"] == pytest.approx(3 * 1.4e7)  # per call = 3 dispatches
    assert b["hbm_over_alg"] == pytest.approx(3 * 1.4e7 / 4e7)
    assert b["f64_tflops"] == pytest.approx(3 * 3e11 / 2e-3 / 1e12, rel=1e-3)
    # a record whose dispatch count per step differs from the profiled one gives no figures
    pmc["per_kernel"]["b"]["launches"] = 16
    b = bench.kernel_table(_FakeEngine(raw), pmc, 2)["b"]
    assert b["hbm_bytes_per_launch"] is None and b["pmc_dispatches_mismatch"]["pmc_per_step"] == 16


def test_dominant_roofline_picks_the_largest_share():
    """The line's roofline is the dominant kernel class's (largest share of the profiled kernel
    time); its achieved rate is algorithmic bytes per call over the call's average duration, and
    its traffic is the PMC record's per-call bytes only where the record measured that class."""
    raw = {"a": [20, 2.0, 20 * 1e6, 20], "b": [8, 16.0, 8 * 4e7, 24]}
    pmc = {"head": "abc", "csrc_sha16": "0" * 16,
           "per_kernel": {"b": {"launches": 12, "hbm_bytes_per_launch": 1.4e7}}}
    t = bench.kernel_table(_FakeEngine(raw), pmc, 2)
    r = bench.dominant_roofline(t, 2, pmc)
    assert r["kernel"].startswith("b") and r["frac"] == t["b"]["frac"]
    assert r["achieved"] == pytest.approx(4e7 / 2e-3 / 1e9, rel=1e-3)  # 4e7 B per 2 ms call
    assert r["traffic"] == pytest.approx(3 * 1.4e7) and r["traffic_head"] == "abc"
    assert r["launches"] == 8
    r = bench.dominant_roofline(bench.kernel_table(_FakeEngine(raw), {}, 2), 2, {})
    assert r["traffic"] is None and r["traffic_head"] is None
    assert bench.dominant_roofline(None, 2, {})["frac"] is None


def test_dominant_class_over_two_instantiations():
    """ks_rows_fin launches two instantiations of one kernel template (228 product
    launches of ~0.94 ms and 4 plain ones of ~6.8 ms per step).  The table keeps them apart
    (each compares with its own rocprof symbol average); the headline class figure is the sum of
    bytes over the sum of time, and lists every instantiation's own figures."""
    steps = 2
    raw = {"ks_rows_fin.prod": [2 * 228, 2 * 228 * 0.9366, 2 * 228 * 5.0e9, 2 * 228],
           "ks_rows_fin.ks": [2 * 4, 2 * 4 * 6.848, 2 * 4 * 3.6e10, 2 * 4],
           "ntt_fwd_cols": [2 * 1328, 2 * 1328 * 0.1739, 2 * 1328 * 4.457e8, 2 * 1328]}
    pmc = {"head": "h", "csrc_sha16": "0" * 16,
           "per_kernel": {"ks_rows_fin.prod": {"launches": 228, "hbm_bytes_per_launch": 5.4e9},
                          "ks_rows_fin.ks": {"launches": 4, "hbm_bytes_per_launch": 3.8e10}}}
    t = bench.kernel_table(_FakeEngine(raw), pmc, steps)
    assert t["ks_rows_fin.prod"]["class"] == "ks_rows_fin"
    assert t["ks_rows_fin.prod"]["avg_us"] == pytest.approx(936.6)
    assert t["ks_rows_fin.ks"]["avg_us"] == pytest.approx(6848.0)
    assert t["ks_rows_fin.prod"]["frac"] == pytest.approx(5.0e9 / 936.6e-6 / 8e12, rel=1e-3)
    r = bench.dominant_roofline(t, steps, pmc)
    assert r["kernel"].startswith("ks_rows_fin:")
    ms = 228 * 0.9366 + 4 * 6.848
    by = 228 * 5.0e9 + 4 * 3.6e10
    assert r["avg_launch_us"] == pytest.approx(ms / 232 * 1e3, rel=1e-4)
    assert r["achieved"] == pytest.approx(by / (ms * 1e-3) / 1e9, rel=1e-3)
    assert r["frac"] == pytest.approx(by / (ms * 1e-3) / 8e12, rel=1e-3)
    assert r["launches"] == 2 * 232
    assert set(r["instantiations"]) == {"ks_rows_fin.prod", "ks_rows_fin.ks"}
    assert r["instantiations"]["ks_rows_fin.ks"]["avg_us"] == pytest.approx(6848.0)
    assert r["traffic"] == pytest.approx((228 * 5.4e9 + 4 * 3.8e10) / 232, rel=1e-6)
    # one instantiation without a PMC figure: no class traffic (never a partial sum)
    del pmc["per_kernel"]["ks_rows_fin.ks"]
    r = bench.dominant_roofline(bench.kernel_table(_FakeEngine(raw), pmc, steps), steps, pmc)
    assert r["traffic"] is None


def test_headline_is_the_dominant_class_not_instantiation():
    """the round-5 profile's largest single symbol was the column pass
    (21.7 %), while the key-switch finishing class summed two instantiations to 22.3 %.  The line's
    headline roofline is the CLASS with the largest share; the largest single instantiation is
    reported beside it under largest_instantiation."""
    steps = 1
    raw = {"ks_rows_fin.prod": [228, 228 * 0.9257, 228 * 5.0e9, 228],
           "ks_rows_fin.ks": [4, 4 * 6.976, 4 * 3.6e10, 4],
           "ntt_fwd_cols": [1328, 1328 * 0.1737, 1328 * 4.457e8, 1328]}
    t = bench.kernel_table(_FakeEngine(raw), {}, steps)
    r = bench.dominant_roofline(t, steps, {})
    assert r["kernel"].startswith("ks_rows_fin:")
    assert r["selected_by"].startswith("class")
    big = r["largest_instantiation"]
    assert big["name"] == "ntt_fwd_cols" and big["class"] == "ntt_fwd_cols"
    assert big["share_of_kernel_time"] > t["ks_rows_fin.prod"]["share_of_kernel_time"]
    assert big["share_of_kernel_time"] < r["share_of_kernel_time"]
    assert big["frac"] == t["ntt_fwd_cols"]["frac"]
