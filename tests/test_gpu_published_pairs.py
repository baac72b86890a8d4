"""The engine against the reference's published CSI curves, calibrated by the reference's own
re-runs (VERDICT r5 "what's weak" 3: the CSI groups had loose z bounds because their
stopping rule is not known).

Three-cornered hat (tools/published_families.py tch): the step-1 CSI files (csi1) re-run the
0.5-dB CSI files (csi) at eps 0 .. 0.4 over LoS, for CNC and MCNC -- 10 pairs of independent
published runs of the same quantities.  With the engine as the third estimate, the pairwise
differences give each run's variance against its stated stopping rule (k_a, k_b) and the
engine's squared bias beta in units of the published sigma, with no stopping-rule assumption
in beta (CPU tests of the solver: tests/test_published_data.py).

* Every pair: beta consistent with 0 at 2 standard errors; pooled over the 10 pairs (inverse
  variance): the engine's bias rms is below 0.35 of one published run's sigma at 2 standard
  errors (measured: 0.28, profiles/r06/pairs/).  A point with the same grid index in both files
  (Eb/N0 5 dB) is not used: its per-point seeds may coincide.
* Calibrated curves: each family's scatter factor (the pairs' median k per receiver; the csi1
  CNC runs scatter as a ~1e7-bit cap would make them, k ~3) scales its published sigma, and the
  curves are held to the FIT bounds of tests/test_gpu_published_families.py, relaxed for the
  uncertainty of k itself (~20 %, so |z| up to ~10 % larger): max |z| <= 5, >= 80 % within 2.
  Replaces that file's CSI_CNC (mean z^2 <= 3) and CSI1_BIAS (mean z^2 <= 12) groups.
* CSI1_WIDE: the CNC LoS eps 0.6 / 0.7 step-1 runs (the driver's commented-out extension)
  scatter 3.5x more than even the calibrated factor (n_eff ~200 trials): no bias (median
  |rel| <= 0.1 %, every row within +-2 %), mean z^2 <= 4 under the calibrated sigma.
* Not compared: CNC LoS eps 0.18 (tests/test_published_data.py: not an eps-0.18 run).
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

import published_families as pf  # noqa: E402

pytestmark = pytest.mark.gpu

PAIRS = pf.pairs()


@pytest.fixture(scope="module")
def pair_results():
    return [pf.tch(p) for p in PAIRS]


@pytest.mark.parametrize("i", range(len(PAIRS)), ids=[p["name"] for p in PAIRS])
def test_published_pair_engine_unbiased(pair_results, i):
    r = pair_results[i]
    print({k: v for k, v in r.items() if k not in ("a", "b")})
    assert r["points"] >= 15 and r["cells"] >= 120  # (Eb/N0 5 dB, index 0 in both grids, not used)
    # each published run's scatter against its rule is a real, finite variance
    assert 0.1 <= r["k_a"] <= 8 and 0.1 <= r["k_b"] <= 8
    assert r["beta"] - 2 * r["se_beta"] <= 0.0, r


def test_published_pairs_pooled_bias(pair_results):
    b = np.array([r["beta"] for r in pair_results])
    w = 1.0 / np.array([r["se_beta"] for r in pair_results]) ** 2
    beta, se = float((b * w).sum() / w.sum()), float(1.0 / np.sqrt(w.sum()))
    print("pooled beta %.4f se %.4f -> bias rms <= %.3f sigma at 2 se" % (beta, se, np.sqrt(max(0.0, beta + 2 * se))))
    assert beta + 2 * se <= 0.12


CAL_EXCLUDED = {"csi1_cnc_los_nant64_eps0.18"}
CSI1_WIDE = {"csi1_cnc_los_nant64_eps0.60", "csi1_cnc_los_nant64_eps0.70"}
CAL_CASES = [c for c in pf.CURVES if pf.curve_name(c) not in CAL_EXCLUDED and
             ((c["family"] == "csi" and c["receiver"] == "cnc") or
              (c["family"] == "csi1" and (c["receiver"] == "cnc" or c["channel"] == "rayleigh")))]


@pytest.mark.parametrize("c", CAL_CASES, ids=[pf.curve_name(c) for c in CAL_CASES])
def test_published_curve_calibrated(pair_results, c):
    k = pf.scatter_factors(pair_results)[(c["family"], c["receiver"])]
    out, _ = pf.measure(c, k_ref=k)
    name = pf.curve_name(c)
    print(name, "k_ref %.3f" % k, {kk: v for kk, v in out.items() if kk not in ("z_map", "file")})
    assert out["compared"] >= 100
    assert out["min_p_zero"] >= 1e-3
    if name in CSI1_WIDE:
        assert out["median_abs_rel"] <= 0.001
        assert out["mean_z2"] <= 4.0 and out["frac_abs_z_le2"] >= 0.75
        for row, rel in out["row_mean_rel"].items():
            assert abs(rel) <= 0.02, (row, rel)
        return
    assert out["median_abs_rel"] <= 0.03
    assert out["frac_abs_z_le1"] >= 0.5 and out["frac_abs_z_le2"] >= 0.8
    assert out["mean_z2"] <= 1.8 and out["max_abs_z"] <= 5.0
    for row, mz in out["row_mean_z"].items():
        assert abs(mz) <= 2.0, (row, mz)
    if c["family"] == "csi":  # the 0.5-dB CNC runs: no bias beyond 0.75 % on any counter row
        for row, rel in out["row_mean_rel"].items():
            assert abs(rel) <= 0.0075, (row, rel)
