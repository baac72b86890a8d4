"""The multi-GPU deal of BASELINE config 4's grid against measured per-point work (VERDICT r4
item 3).  profiles/r05/grid/c4_points_{rayleigh,los}.json are one-GPU records of the
915-point grid (tools/grid_record.py): the trials the stopping rule ran at every point.  Every
point of a stopping-rule round shares one launch and the same per-trial work, so trials ARE
the per-point cost.  sweep.point_costs must rank the points like the measurement, and the
LPT deal it drives must balance the MEASURED work at N = 2, 4, 8."""
import json
import os

import numpy as np
import pytest
from scipy.stats import spearmanr

import sweep

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RECORDS = {ch: os.path.join(REPO, "profiles", "r05", "grid", f"c4_points_{ch}.json") for ch in ("rayleigh", "los")}


def _record(ch):
    with open(RECORDS[ch]) as f:
        return json.load(f)


def _model(d, ch):
    return sweep.point_costs(np.asarray(d["ibo"]), np.asarray(d["ebn0"]), d["bits_per_symbol"], 64, d["n_err_min"],
                             d["bits_sent_max"], d["iters"], 64, False, ch)


@pytest.mark.parametrize("ch", sorted(RECORDS))
def test_cost_model_ranks_points_like_the_measurement(ch):
    d = _record(ch)
    trials = np.asarray(d["trials_per_point"], dtype=np.float64)
    assert trials.size == 915 and trials.sum() > 200000
    rho = spearmanr(_model(d, ch), trials).correlation
    print(ch, "rank correlation", rho)
    assert rho >= 0.9


@pytest.mark.parametrize("ch", sorted(RECORDS))
@pytest.mark.parametrize("n", [2, 4, 8])
def test_lpt_deal_balances_measured_work(ch, n):
    """Points dealt by the model (what run_grid does), loads evaluated on the measured trials:
    the busiest rank carries <= 1.10 x the mean."""
    d = _record(ch)
    trials = np.asarray(d["trials_per_point"], dtype=np.float64)
    costs = _model(d, ch)
    loads = [trials[sweep.owned_points(trials.size, r, n, costs)].sum() for r in range(n)]
    assert sum(len(sweep.owned_points(trials.size, r, n, costs)) for r in range(n)) == trials.size
    print(ch, n, "max / mean", max(loads) / np.mean(loads))
    assert max(loads) <= 1.10 * np.mean(loads)


def test_cost_model_pilot_floor_and_distortion():
    """Model properties: no point below the stopping rule's pilot batch; at a fixed Eb/N0 a
    lower IBO (more clipping) never costs more trials over LoS; Rayleigh sees 1/A of it."""
    ibo, ebn0 = np.arange(0, 7.01, 0.5), np.arange(0, 30.01, 0.5)
    c_los = sweep.point_costs(ibo, ebn0, 12288, 64, 1e5, 5e6, [0], 64, False, "los").reshape(len(ibo), -1)
    c_ray = sweep.point_costs(ibo, ebn0, 12288, 64, 1e5, 5e6, [0], 64, False, "rayleigh").reshape(len(ibo), -1)
    per_trial = 64
    assert c_los.min() >= 64 * per_trial and c_ray.min() >= 64 * per_trial
    assert np.all(np.diff(c_los, axis=0) >= -1e-9)
    assert np.all(c_ray >= c_los - 1e-9)
    assert sweep.soft_limiter_sdr(0.0) < sweep.soft_limiter_sdr(3.0) < sweep.soft_limiter_sdr(7.0)
