"""The engine against four more families of the reference's published BER curves
(VERDICT r4 item 1): channel-estimation error (CSI eps; the step-1 runs over LoS and
Rayleigh as a fourth family), BER vs IBO including the noiseless Eb/N0 = 1000 dB runs, and
single-antenna arrays.  tools/published_families.py holds the
machinery (each driver's own stopping rule -> sigma of the published value; the engine's
per-trial spread -> its own sigma); profiles/r05/families/ the measured statistics and z maps.

The engine's counts are deterministic (fixed seeds, exact kernel), so these statistics are
the same on every box.  Groups:

* FIT -- the bounds of test_published_curve_paper_config (>= 50 % of the points within 1
  sigma, >= 85 % within 2, mean z^2 <= 1.8, max |z| <= 4.5, median |rel| <= 3 %), plus
  no counter row whose mean z leaves +-2: MCNC with CSI error (5 eps), BER vs IBO over
  LoS at Eb/N0 15 and 1000 (CNC, MCNC), over Rayleigh (CNC, MCNC) and two-path (MCNC) at
  64 antennas, and the 1-antenna LoS / two-path curves (CNC, MCNC).
* CNC with CSI error (0.5-dB runs) and the step-1 CNC / Rayleigh-MCNC CSI runs: their scatter
  exceeds the stated stopping rule's, so they are compared in tests/test_gpu_published_pairs.py
  with a published sigma calibrated by the reference's own re-runs (three-cornered hat).
* FIT also holds the BER-vs-Eb/N0 curves at IBO 1 (the committed drivers' own setting) and
  IBO 0 (family ebn0: LoS, two-path, Rayleigh x CNC, MCNC) and 32 more BER-vs-IBO files
  (family ibo2: Eb/N0 10-20 and 1000 dB, IBO -9..9 included; row layout read from the data,
  published_families.layout).  FIT_LOWCOUNT: two ibo2 files at Eb/N0 18 whose z statistics fit
  (mean z^2 ~1) but whose few-error points put the median |rel| at 3-4 %: the FIT z bounds with
  a 5 % median.  The noiseless ibo2 files (IBO down to -9 dB) hold float32 to >= 99.7 %.
* FIT also: the 1-antenna LoS / two-path BER-vs-Eb/N0 curves at IBO 0 (family small2, CNC);
  FIT_OUTLIER: their MCNC files (0.5-dB steps), the FIT bounds but for max |z|: at most one isolated
  point each (z -14 at iteration 5, 18.5 dB; the no-distortion row at 8 dB, z 6.5).  Not
  compared in small2: the 1-antenna Rayleigh and 4-antenna curves (as in the IBO families),
  the 16-antenna files (5 points), LoS IBO 50 (its no-distortion row reads BER 0.79-0.83, a
  broken clean run; its distorted rows agree within 0.6 %) and two-path IBO 20 (5-18 % apart).
* Not compared (the z maps in profiles/r05/families/).  Every exclusion but one
  is backed by the published files alone, in tests/test_published_data.py (CPU): the CNC LoS /
  two-path IBO 0..8 files (below every other run of the same quantities), the 4-antenna LoS /
  two-path curves (outside the band of the agreeing 1- and 64-antenna curves), the TOI family
  (distortion ordered against the stated TOIs), the 1-antenna Rayleigh curves (below the
  independent-channel closed form: the replayed channel sequence), two-path IBO 20 (iterations
  unequal to the standard RX where nothing clips), LoS IBO 50 (a clean row worse than
  guessing), the 16-antenna pair (CNC and MCNC disagree on the standard RX) and CNC LoS eps 0.18
  (out of order).  Parity unresolved: the 4-antenna Rayleigh curves (no band to test against).

Noiseless runs: where the reference published BER 0 (no erroneous symbol in its trials),
the engine's fraction q of erroneous trials must make that likely, (1 - q)^n_ref >= 1e-3;
and the float32 instance agrees with float64 on >= 99.9 % of the (trial, counter) entries.
"""
import sys
import os

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

import published_families as pf  # noqa: E402

pytestmark = pytest.mark.gpu

NOT_COMPARED = {"ibo_cnc_two_path_nant64_ebn0_15", "small_cnc_rayleigh_nant1_ebn0_15",
                "small_mcnc_rayleigh_nant1_ebn0_15", "csi1_cnc_los_nant64_eps0.18",
                "ibo2_cnc_los_nant64_ebn0_15_ibo0_8_0.5"}
FIT_LOWCOUNT = {"ibo2_cnc_los_nant64_ebn0_18_ibo0_9_0.25", "ibo2_cnc_two_path_nant64_ebn0_18_ibo0_9_0.25"}


def _group(c):
    name = pf.curve_name(c)
    if c["n_ant"] == 4 or name in NOT_COMPARED or c["family"] == "toi":
        return None
    if c["family"] == "small2":  # the 1-antenna LoS / two-path BER-vs-Eb/N0 curves at IBO 0
        if c["n_ant"] != 1 or c["channel"] == "rayleigh" or c["ibo"] != 0:
            return None
        return "fit" if c["receiver"] == "cnc" else "fit_outlier"
    if c["family"] == "csi" and c["receiver"] == "cnc":
        return None  # calibrated by the published re-runs: tests/test_gpu_published_pairs.py
    if c["family"] == "csi1" and (c["receiver"] == "cnc" or c["channel"] == "rayleigh"):
        return None  # likewise
    if name in FIT_LOWCOUNT:
        return "fit_lowcount"
    return "fit"


CASES = [c for c in pf.CURVES if _group(c)]


@pytest.mark.parametrize("c", CASES, ids=[pf.curve_name(c) for c in CASES])
def test_published_family_curve(c):
    noiseless = c.get("ebn0") == 1000.0
    out, _ = pf.measure(c, f32_check=noiseless)
    print(pf.curve_name(c), {k: v for k, v in out.items() if k not in ("z_map", "file")})
    g = _group(c)
    assert out["compared"] >= 20
    assert out["median_abs_rel"] <= (0.05 if g == "fit_lowcount" else 0.03)
    if g in ("fit", "fit_lowcount", "fit_outlier"):
        assert out["frac_abs_z_le1"] >= 0.5 and out["frac_abs_z_le2"] >= 0.85
        assert out["mean_z2"] <= 1.8 and (g == "fit_outlier" or out["max_abs_z"] <= 4.5)
        if g == "fit_outlier":  # exactly the one isolated point the docstring names leaves 4.5
            far = [v for row in out["z_map"] for v in row if v is not None and abs(v) > 4.5]
            assert len(far) <= 1, far
        for row, mz in out["row_mean_z"].items():
            assert abs(mz) <= 2.0, (row, mz)
    # zero region: published 0 must be likely under the engine's rate of erroneous trials
    assert out["min_p_zero"] >= 1e-3
    if noiseless and c["family"] == "ibo":
        assert out["zero_points"] >= 100
        assert out["f32_entry_agreement"] >= 0.999
        assert out["f32_mean_z2"] <= 1.8
    elif noiseless:  # ibo2: down to IBO -9 dB, where float32 flips a few more decisions
        assert out["f32_entry_agreement"] >= 0.997
        assert out["f32_mean_z2"] <= 1.8
