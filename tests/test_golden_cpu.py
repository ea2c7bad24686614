"""Oracle freeze: the CPU restatement must reproduce the
committed fixtures tests/golden/{dpgo,lcd}_small.npz (made by
tests/golden/make_golden.py). A change to oracle/ that moves any restated
result fails here, so the oracle cannot co-evolve with the kernels unseen.

Integers (tCG counts, accept flags, inlier masks, RANSAC iterations) must be
identical; floats identical up to 1e-12 relative (the oracle is built with
-ffp-contract=off; the slack only absorbs a different libm on another host)."""
import sys
from pathlib import Path

import numpy as np
import pytest

GOLD = Path(__file__).resolve().parent / "golden"
sys.path.insert(0, str(GOLD))
import make_golden as MG  # noqa: E402


def _close(a, b, rel=1e-12):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    assert a.shape == b.shape
    scale = np.maximum(1.0, np.abs(b))
    same_nan = np.isnan(a) & np.isnan(b)
    assert np.all(same_nan | (np.abs(a - b) <= rel * scale)), np.nanmax(np.abs(a - b) / scale)


def test_dpgo_fixture_reproduced():
    d = np.load(GOLD / "dpgo_small.npz")
    g = MG.graph_from(d)
    out = MG.run_dpgo_oracle(g, int(d["r"]), d["X0"])
    assert np.array_equal(out["round_ints"], d["round_ints"])
    _close(out["round_f"], d["round_f"])
    assert np.array_equal(out["mu"], d["mu"])
    _close(out["weights"], d["weights"])
    _close(out["X_final"], d["X_final"])
    # the fixture exercises the GNC schedule: three weight updates, some outliers down-weighted
    assert d["weights"].shape[0] == 3 and (d["weights"][-1] < 0.5).any()


@pytest.mark.parametrize("k", range(len(MG.LCD_CASES)))
def test_lcd_fixture_reproduced(k):
    d = np.load(GOLD / "lcd_small.npz")
    pool = MG.pool_from(d)
    case = MG.LCD_CASES[k]
    assert d["cases"][k].tolist() == [case[0], case[1] == "gcc11", case[2] == "hamming", case[3]]
    ints, T, masks = MG.run_lcd_oracle(pool, case)
    assert np.array_equal(ints, d[f"ints_{k}"])
    assert np.array_equal(masks, d[f"masks_{k}"])
    _close(T, d[f"T_{k}"])
    assert ints[0::2, 4].sum() >= 7 and ints[1::2, 4].sum() == 0  # planted pairs accepted, random pairs not


def test_generator_inputs_unchanged():
    """The fixtures carry their inputs; the synthetic generators still make
    the same ones (so GPU tests on generator output and the fixtures agree)."""
    d = np.load(GOLD / "dpgo_small.npz")
    g, P, X0 = MG.dpgo_inputs()
    assert np.array_equal(g.r1, d["r1"]) and np.array_equal(g.R, d["R"]) and np.array_equal(X0, d["X0"])
    l = np.load(GOLD / "lcd_small.npz")
    pool = MG.lcd_inputs()
    assert np.array_equal(pool.desc, l["desc"]) and np.array_equal(pool.bearings, l["bearings"])
