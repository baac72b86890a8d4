"""BASELINE config 4 on the GPU: the paper's fixed-BER grid (IBO 0..7.5 x Eb/N0 10..22 dB,
64 antennas, N_fft 4096, 2048 sub-carriers, 64-QAM, receiver iterations 0..8, no clean
run, bits_sent_max 5e6, n_err_min 1e5; main_mp_miso_cnc_constant_ber_req_ebn0_vs_ibo.py:
100-215) through sweep.run_grid, against the reference's published grids
(tests/golden/published_fixed_ber1.0e-02_*.csv, data files of its figs/csv_results).

Compared at every (point, iteration) with published BER >= 1e-3 (tools/fixed_ber_check.py):
* no bias: the mean relative difference of every iteration is within 1 % (measured
  <= 0.3 %);
* median relative difference <= 2 % (measured 0.75-1.0 %);
* z-scores: the published value's sigma from 16 replicas of the reference's estimator at
  its stopping-rule trial counts (per counter: a counter closes at n_err_min errors or the
  bit budget), the GPU estimate's from the same spread at its own trial counts.  Measured
  (profiles/r03/stats/config4_sigma.log): 47-58 % within 1 sigma, 82-85 % within 2,
  p95 |z| 2.9-3.1, mean z^2 2.0-2.5 -- about 1.4x the spread the replicas predict.  The
  replica sigma is right for this estimator (one replica against the other 15: 67 % within
  1 sigma, 94 % within 2; profiles/r03/stats/config4_self_check.log), so the excess is in
  the published estimates.  Round 4 located it (spread statistics below): a random shift
  per point, shared by the point's 9 counters, independent between neighbouring points,
  with no signed mean in any iteration or IBO row; the published BER-vs-Eb/N0 curves show
  plain 1-sigma statistics (tests/test_gpu_link.py).  Bounds:
  >= 75 % within 2 sigma, p95 |z| <= 3.5, mean z^2 <= 3, max |z| <= 8; the replica
  self-check >= 90 % within 2 sigma;
* round 6: the reference published the CNC grids twice; a three-cornered hat over the two
  runs and the engine measures each run's scatter (~3x the replica prediction, both runs
  alike) and the engine's bias (consistent with 0) without any stopping-rule assumption
  (test_fixed_ber_published_pair);
* the derived curve itself (Eb/N0 needed for BER 1e-2 per IBO and iteration): reachable
  exactly where the published grid reaches it, mean |difference| <= 0.1 dB (measured
  0.01-0.05 dB).
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("receiver,channel", [("cnc", "rayleigh"), ("cnc", "los"), ("cnc", "two_path"),
                                              ("mcnc", "rayleigh")])
def test_fixed_ber_grid_vs_published(receiver, channel):
    import fixed_ber_check
    out, ber, pub, z = fixed_ber_check.run(channel, receiver, "f64")
    print(out)
    assert out["points"] == 400 and out["compared"] > 1000
    assert out["max_abs_bias_per_iteration"] <= 0.01
    assert out["median_rel"] <= 0.02
    assert out["frac_abs_z_le2"] >= 0.75 and out["p95_abs_z"] <= 3.5
    assert out["mean_z2"] <= 3.0 and out["max_abs_z"] <= 8.0
    assert out["replica_self_check"]["frac_abs_z_le2"] >= 0.9
    r = out["req_ebn0_at_ber_1e2"]
    assert r["finite_mismatch"] == 0 and r["compared"] >= 70 and r["mean_abs_db"] <= 0.1
    # where the excess spread sits (tools/fixed_ber_check.py spread_stats,
    # round-4 record profiles/r04/config4/config4_spread.json): the 9 counters of a point move
    # together (z of consecutive iterations correlated 0.92-0.98), no iteration column and no
    # IBO row carries a mean z beyond 3 sigma of its own scatter, and the point z of
    # neighbouring Eb/N0 points are uncorrelated (lag-1 -0.11 ... +0.03) -- no region-confined
    # or smooth signed mismatch; the excess is a per-point random shift (point-z variance
    # 1.7-2.4 instead of 1, most at budget-limited points)
    sp = out["spread"]
    assert sp["within_point_corr"] >= 0.85
    assert sp["iterations_outside"] == 0 and sp["rows_outside"] == 0, sp
    assert abs(sp["lag1_point_z_along_ebn0"]) <= sp["lag1_bound"], sp


@pytest.mark.parametrize("receiver,channel,n_ant,ibo_step", [
    ("mcnc", "los", 64, 0.5), ("mcnc", "two_path", 64, 0.5),
    ("cnc", "los", 64, 0.25), ("cnc", "rayleigh", 64, 0.25), ("cnc", "two_path", 64, 0.25),
    ("cnc", "los", 1, 0.5), ("cnc", "two_path", 1, 0.5), ("mcnc", "los", 1, 0.5), ("mcnc", "two_path", 1, 0.5)])
def test_fixed_ber_grid_more_published(receiver, channel, n_ant, ibo_step):
    """Nine more fixed-BER grids the reference publishes (round 5, profiles/r05/config4/): the
    MCNC LoS / two-path paper grids, the CNC grids at 0.25-dB IBO steps (800 points) and the
    1-antenna LoS / two-path grids.  The bounds above, except that an iteration column may
    carry a small signed shift (|mean z| <= 0.35 instead of 3 / sqrt(n): MCNC LoS iteration 1
    at -0.31 z, MCNC two-path iterations 6-8 at +0.24 ... +0.30 z, at most 0.5 % relative) and
    the MCNC two-path grid reaches BER 1e-2 at one (IBO, iteration) cell the published grid
    does not.  The 1-antenna Rayleigh grids are left out: their point z correlate along Eb/N0
    (lag-1 0.70 / 0.81), the reference's one replayed channel sequence."""
    import fixed_ber_check
    out, ber, pub, z = fixed_ber_check.run(channel, receiver, "f64", n_ant=n_ant, ibo_step=ibo_step)
    print(out)
    assert out["points"] == int(round(8 / ibo_step)) * 25 and out["compared"] > 1000
    assert out["max_abs_bias_per_iteration"] <= 0.01
    assert out["median_rel"] <= 0.02
    assert out["frac_abs_z_le2"] >= 0.75 and out["p95_abs_z"] <= 3.5
    assert out["mean_z2"] <= 3.0 and out["max_abs_z"] <= 8.0
    assert out["replica_self_check"]["frac_abs_z_le2"] >= 0.9
    r = out["req_ebn0_at_ber_1e2"]
    assert r["finite_mismatch"] <= 1 and r["compared"] >= 70 and r["mean_abs_db"] <= 0.1
    sp = out["spread"]
    assert sp["within_point_corr"] >= 0.85 and sp["rows_outside"] == 0, sp
    assert max(abs(c["mean_z"]) for c in sp["iterations"]) <= 0.35, sp
    assert abs(sp["lag1_point_z_along_ebn0"]) <= sp["lag1_bound"], sp


def test_fixed_ber_grid_baseline_extent():
    """BASELINE config 4 at its stated extent (Eb/N0 0..30 x IBO 0..7 dB, 0.5 dB steps =
    915 points, CNC 0..8) on one GPU: every counter of every point closed
    by the stopping rule, the standard receiver's BER non-increasing in Eb/N0 at every IBO,
    and the sub-grid shared with the published grid in line with it."""
    import fixed_ber_check
    out, ber = fixed_ber_check.run_baseline("rayleigh", "cnc", "f64")
    print(out)
    assert out["points"] == 915 and out["all_counters_closed"]
    assert out["standard_rx_ber_rises"] == 0
    sh = out["shared_with_published"]
    assert sh["points"] == 375 and sh["compared"] > 1000 and sh["median_rel"] <= 0.02


@pytest.fixture(scope="module")
def config4_pairs():
    import fixed_ber_check
    return {ch: fixed_ber_check.pair_check(ch) for ch in ("rayleigh", "los", "two_path")}


@pytest.mark.parametrize("channel", ["rayleigh", "los", "two_path"])
def test_fixed_ber_published_pair(config4_pairs, channel):
    """The reference published each CNC grid twice (0.5- and 0.25-dB IBO steps, independent
    runs at the IBO values they share, IBO 0 left out: tools/fixed_ber_check.py pair_check).
    Three-cornered hat with the engine as the third estimate (round 6): the engine's squared
    bias beta is consistent with 0, and the two published runs scatter alike, ~3x the variance
    the replicas of the stated stopping rule give (measured k 2.9-4.0) -- the config-4 excess
    of the z statistics above is in the published estimates, measured from their own
    disagreement."""
    r = config4_pairs[channel]
    print(r)
    assert r["points"] >= 250 and r["cells"] >= 1500
    assert r["beta"] - 2 * r["se_beta"] <= 0.0, r
    assert 1.5 <= r["k_a"] <= 6 and 1.5 <= r["k_b"] <= 6, r
    assert abs(r["k_a"] - r["k_b"]) <= 3 * (r["se_k_a"] ** 2 + r["se_k_b"] ** 2) ** 0.5, r


def test_fixed_ber_published_pairs_pooled(config4_pairs):
    b = np.array([r["beta"] for r in config4_pairs.values()])
    w = 1.0 / np.array([r["se_beta"] for r in config4_pairs.values()]) ** 2
    beta, se = float((b * w).sum() / w.sum()), float(1.0 / np.sqrt(w.sum()))
    print("config-4 pooled beta %.4f se %.4f -> bias rms <= %.3f published sigma at 2 se"
          % (beta, se, np.sqrt(max(0.0, beta + 2 * se))))
    assert beta + 2 * se <= 0.4
