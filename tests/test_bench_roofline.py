"""bench.py's roofline fields from the committed PMC summaries (no GPU): the cycle-based VALU-busy fraction
(SQ_ACTIVE_INST_VALU quad-cycles x 4 over the SIMD-cycles, GRBM_GUI_ACTIVE summed over the 8 XCDs) and the
limiter `bound` (the largest of the HBM, atomic-request and VALU fractions, or latency below one half)."""
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_bound_takes_the_largest_fraction():
    assert bench.bound_of(0.46, 0.29, 0.635) == "valu"      # C4
    assert bench.bound_of(0.33, 0.86, 0.76) == "atomic"     # C3
    assert bench.bound_of(0.70, 0.20, None) == "hbm"
    assert bench.bound_of(0.30, 0.20, 0.40) == "latency"


def test_valu_busy_from_the_pmc_counters(tmp_path, monkeypatch):
    # one launch of 1e6 cycles per XCD on 1,024 SIMDs, the VALU issuing in a quarter of them
    d = {"traffic_bytes_per_launch": 1e9, "source": "synthetic", "valu_insts_per_launch": 2.5e8,
         "grbm_gui_active_per_launch": 8e6, "valu_active_quads_per_launch": 0.25 * 1024 * 1e6 / 4,
         "inst_active_quads_per_launch": 0.5 * 1024 * 1e6 / 4}
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "pmc_cx.json").write_text(json.dumps(d))
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    t = bench.pmc_traffic("cx")
    assert t["valu_busy"] == pytest.approx(0.25)
    assert t["inst_busy"] == pytest.approx(0.5)
    assert bench.pmc_traffic("missing") is None


@pytest.mark.parametrize("config", ["c2", "c3", "c4", "c5"])
def test_committed_pmc_summaries_give_a_valu_busy_fraction(config):
    t = bench.pmc_traffic(config)
    assert t is not None and 0.2 < t["valu_busy"] < 1.0, t
