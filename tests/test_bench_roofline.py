"""bench.py's roofline object (the bench contract's `roofline`): on the
committed PMC rates (profiles/pmc_rates.json) and a synthetic set of stage
times, the dominant stage carries bound / achieved / peak / unit / frac /
traffic with frac = achieved / peak, and every stage entry has a bound.
Host logic only: no GPU."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def test_roofline_fields_and_ratio():
    import bench
    rates = bench.pmc_rates()
    if not rates:
        pytest.skip("no committed PMC rates")
    stage_avg = {"prop0": 0.556, "prop1": 0.293, "final": 0.705, "s_grid": 0.628, "sam_head": 0.514}
    roof, stages = bench.rooflines(stage_avg, 512 * 512, 0, rates, timed_clock={"ghz": 2.2})
    assert roof["kernel"] == "final"
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in roof and roof[k] is not None, k
    assert roof["frac"] == pytest.approx(roof["achieved"] / roof["peak"])
    assert 0.0 < roof["frac"] < 1.5
    assert roof["timed_clock_ghz"] == 2.2
    assert set(stages) == set(stage_avg)
    for st, e in stages.items():
        assert "bound" in e and e["frac"] > 0, st
