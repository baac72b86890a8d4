"""The engine against six more families of BER curves the reference publishes.

Families (CSV data files of figs/csv_results, copied to tests/golden as published_*.csv; row
layout axis, no-distortion, standard RX, CNC / MCNC iterations 1..8):

* ``csi``   -- BER vs Eb/N0 (5..20 dB, 0.5 dB) with channel-estimation error eps in
  {0, 0.1, 0.2, 0.3, 0.4}: LoS, 64 antennas, soft limiter at IBO 0 dB, F 4096 / S 2048.
  Driver main_mp_miso_cnc_csi_err_ber_vs_ebn0.py:41-63,119 (bits_sent_max 3e7, n_err_min
  1e7) and main_mp_miso_mcnc_csi_err_ber_vs_ebn0.py (n_err_min 1e6).
* ``ibo``   -- BER vs IBO (0..9 dB, 0.5 dB) at Eb/N0 15 dB and 1000 dB (the noiseless
  runs), LoS, 64 antennas; plus the Rayleigh / two-path curves at Eb/N0 15 (IBO 0..8.5).
  Driver main_mp_miso_cnc_ber_vs_ibo.py:41-58,105 (bits_sent_max 1e7, n_err_min 1e5) and
  main_mp_miso_mcnc_ber_vs_ibo.py (same settings).
* ``csi1``  -- BER vs Eb/N0 (5..20 dB, 1 dB) with CSI error: the step-1 runs of the same
  drivers, over LoS (eps 0 .. 0.7, the driver's commented-out extension of csi_epsylon_lst)
  and over Rayleigh (eps 0.01 .. 0.2; chan_lst = [Rayleigh]) -- other revisions of the
  committed drivers, whose stopping rule (3e7 bits, n_err_min 1e7 / 1e6) is assumed
  unchanged.  The LoS eps 0 .. 0.4 curves are independent re-runs of the ``csi`` family's.
* ``ebn0``  -- BER vs Eb/N0 at 64 antennas, LoS / two-path / Rayleigh, CNC and MCNC, at IBO 1 dB
  (5..20 dB, 1 dB: the committed drivers' own setting, main_mp_miso_{cnc,mcnc}_ber_vs_ebn0.py:40-58,
  ibo_arr [1, 3], 1e7 bits, n_err_min 1e6) and at IBO 0 dB (0.5-dB steps, another revision of
  the same drivers, stopping rule assumed unchanged).  The IBO 3 curves are
  tests/test_gpu_link.py's.
* ``ibo2``  -- every other BER-vs-IBO file at 64 antennas: Eb/N0 10, 12, 15, 18, 20 and 1000 dB,
  IBO -9..9 / 0..9 / -3..3 in 0.25-2 dB steps (revisions of main_mp_miso_{cnc,mcnc}_ber_vs_ibo.py,
  stopping rule as the ``ibo`` family's; row layout as that family's, the 10-row files "full").
* ``small2`` -- BER vs Eb/N0 at 1, 4 and 16 antennas (IBO 0, and 1 antenna at IBO 20 / 50):
  the BER-vs-Eb/N0 drivers with other n_ant_arr / ibo_arr (stopping rule assumed as theirs;
  rows [clean, standard RX, the file's iterations]).
* ``toi``   -- BER vs Eb/N0 (5..20 dB, 1 dB) with the third-order PA (TOI 22.75 dB), two-path,
  1 and 4 antennas, CNC and MCNC: main_miso_{cnc,mcnc}_ber_vs_ebn0_toi.py (not the mp Link: the
  drivers inline the loop, 1e7 bits / 1e5 errors).  Their AGC and receivers use one measured
  gain for every antenna, alpha_estimate = mean over 1e4 unprecoded symbols of
  |mean_k(rx_k / clean_k)| (:95-121,247-249): restated by toi_alpha_estimate() and passed as
  mimo_point.array_alpha / cnc_alpha; the array PA's cubic coefficient is set with the
  precoding gain of an unprecoded array (update_distortion before any set_precoding_matrix,
  antenna_array.py:328-360), i.e. for the modem's average sample power.
* ``small`` -- BER vs IBO at 1 and 4 antennas (LoS, Rayleigh, two-path), Eb/N0 15.  The
  same driver with n_ant_arr = [1] / [4] (assumed: the committed driver lists [64]).

The published value's sigma is the spread of the reference's own estimator under its
stopping rule: every counter stops on its own at n_err_min errors or bits_sent_max bits
(mp_model.py:137-138,177-187), so counter c of a point averages
n_c = min(ceil(bits_max / B), ceil(n_err_min / (p_c B))) trials (B = 12,288 bits per OFDM
symbol, p_c the counter's BER).  Trials are independent (LoS / two-path reroll the RX
position per trial from each worker's own generator; the Rayleigh workers' shared channel
sequence changed nothing measurable at 64 antennas, tools/replay_sigma.py), so
sigma_ref = sd_trial / sqrt(n_c), with sd_trial the per-trial BER spread the engine measures
at that point.  sigma_gpu = sd_trial / sqrt(n_tr) by the same token.  Compared: points with
BER >= 1e-5 whose published estimate rests on >= 100 errors.

Zero-region check (the noiseless runs reach BER 0): where the published value is exactly 0,
the reference saw no erroneous symbol in n_c trials.  With q the fraction of the engine's
trials that hold any bit error, that has probability (1 - q)^n_c; a point where that is
below 1e-3 would be a mismatch.

Where the published sigma rests on an assumed stopping rule, the reference's own re-runs
calibrate it: tch() (three-cornered hat over published pairs, below) measures each run's scatter
factor k and the engine's bias without that assumption; measure(k_ref=k) then scales the
published variance (tests/test_gpu_published_pairs.py).

    python tools/published_families.py [--family csi|csi1|ebn0|ibo2|small2|toi|ibo|small|all] [--out file.json]
    python tools/published_families.py --pairs [--out file.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "m-mimo-ofdm-with-nonlinear-pa-sim_amd"), os.path.join(REPO, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

GOLDEN = os.path.join(REPO, "tests", "golden")
ITERS = list(range(9))  # standard RX + CNC / MCNC iterations 1..8 (the drivers' cnc_n_iter_lst)
N_SC, N_FFT, M = 2048, 4096, 64
BPS = N_SC * 6
TAIL = "niter1_2_3_4_5_6_7_8"


def _curves():
    out = []
    for rx, n_err in (("cnc", 1e7), ("mcnc", 1e6)):
        for eps in (0.0, 0.1, 0.2, 0.3, 0.4):
            out.append(dict(family="csi", receiver=rx, channel="los", n_ant=64, axis="ebn0", ibo=0.0, eps=eps,
                            bits_max=3e7, n_err_min=n_err,
                            file="ber_vs_ebn0_%s_los_csi_eps%1.3f_nant64_ibo0_ebn0_min5_max20_step0.50_%s" % (rx, eps, TAIL)))
    for rx, n_err, grid in (("cnc", 1e7, {"los": (0.0, 0.01, 0.1, 0.18, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7),
                                          "rayleigh": (0.01, 0.1, 0.2)}),
                            ("mcnc", 1e6, {"los": (0.0, 0.01, 0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7),
                                           "rayleigh": (0.01, 0.1)})):
        for ch, epss in grid.items():
            for eps in epss:
                out.append(dict(family="csi1", receiver=rx, channel=ch, n_ant=64, axis="ebn0", ibo=0.0, eps=eps,
                                bits_max=3e7, n_err_min=n_err,
                                file="ber_vs_ebn0_%s_%s_csi_eps%1.3f_nant64_ibo0_ebn0_min5_max20_step1.00_%s"
                                % (rx, ch, eps, TAIL)))
    for rx in ("cnc", "mcnc"):
        for ebn0 in (15, 1000):
            out.append(dict(family="ibo", receiver=rx, channel="los", n_ant=64, axis="ibo", ebn0=float(ebn0), eps=None,
                            bits_max=1e7, n_err_min=1e5,
                            file="ber_vs_ibo_%s_los_nant64_ebn0_%d_ibo_min0_max9_step0.50_%s" % (rx, ebn0, TAIL)))
        for ch in ("rayleigh", "two_path"):
            out.append(dict(family="ibo", receiver=rx, channel=ch, n_ant=64, axis="ibo", ebn0=15.0, eps=None,
                            bits_max=1e7, n_err_min=1e5,
                            file="ber_vs_ibo_%s_%s_nant64_ebn0_15_ibo_min0_max8_step0.50_%s" % (rx, ch, TAIL)))
    for ibo, step in ((1, "1.00"), (0, "0.50")):
        for rx in ("cnc", "mcnc"):
            for ch in ("los", "two_path", "rayleigh"):
                out.append(dict(family="ebn0", receiver=rx, channel=ch, n_ant=64, axis="ebn0", ibo=float(ibo), eps=None,
                                bits_max=1e7, n_err_min=1e6,
                                file="ber_vs_ebn0_%s_%s_nant64_ibo%d_ebn0_min5_max20_step%s_%s" % (rx, ch, ibo, step, TAIL)))
    import re
    named = {o["file"] for o in out}
    pat = re.compile(r"ber_vs_ibo_(cnc|mcnc)_(los|rayleigh|two_path)_nant64_ebn0_(\d+)_ibo_min(-?\d+)_max(\d+)_step([\d.]+)_"
                     + TAIL + r"\.csv$")
    ibo_named = {"ber_vs_ibo_%s_los_nant64_ebn0_%d_ibo_min0_max9_step0.50_%s" % (rx, e, TAIL)
                 for rx in ("cnc", "mcnc") for e in (15, 1000)}
    ibo_named |= {"ber_vs_ibo_%s_%s_nant64_ebn0_15_ibo_min0_max8_step0.50_%s" % (rx, ch, TAIL)
                  for rx in ("cnc", "mcnc") for ch in ("rayleigh", "two_path")}
    for f in sorted(os.listdir(GOLDEN)):
        m = pat.match(f[len("published_"):]) if f.startswith("published_") else None
        if not m or f[len("published_"):-4] in named | ibo_named:
            continue
        rx, ch, e, lo, hi, st = m.groups()
        out.append(dict(family="ibo2", receiver=rx, channel=ch, n_ant=64, axis="ibo", ebn0=float(e), eps=None,
                        bits_max=1e7, n_err_min=1e5, ibo_range=(int(lo), int(hi), float(st)), file=f[len("published_"):-4]))
    pat2 = re.compile(r"ber_vs_ebn0_(cnc|mcnc)_(los|rayleigh|two_path)_nant(1|4|16)_ibo(\d+)_ebn0_min(\d+)_max(\d+)"
                      r"_step([\d.]+)_niter([\d_]+)\.csv$")
    for f in sorted(os.listdir(GOLDEN)):
        m = pat2.match(f[len("published_"):]) if f.startswith("published_") else None
        if not m:
            continue
        rx, ch, na, ibo, lo, hi, st, it = m.groups()
        out.append(dict(family="small2", receiver=rx, channel=ch, n_ant=int(na), axis="ebn0", ibo=float(ibo), eps=None,
                        bits_max=1e7, n_err_min=1e6, ebn0_range=(int(lo), int(hi), float(st)), file=f[len("published_"):-4]))
    for rx, na, tag, toi in (("cnc", 1, 22, 22.75), ("cnc", 1, 5, 5.0), ("cnc", 4, 22, 22.75),
                             ("mcnc", 1, 22, 22.75), ("mcnc", 4, 22, 22.75)):
        out.append(dict(family="toi", receiver=rx, channel="two_path", n_ant=na, axis="ebn0", toi=toi, eps=None,
                        bits_max=1e7, n_err_min=1e5,
                        file="toi_ber_vs_ebn0_%s_two_path_nant%d_ibo%d_ebn0_min5_max20_step1.00_%s" % (rx, na, tag, TAIL)))
    for rx in ("cnc", "mcnc"):
        for ch in ("los", "rayleigh", "two_path"):
            for na in (1, 4):
                out.append(dict(family="small", receiver=rx, channel=ch, n_ant=na, axis="ibo", ebn0=15.0, eps=None,
                                bits_max=1e7, n_err_min=1e5,
                                file="ber_vs_ibo_%s_%s_nant%d_ebn0_15_ibo_min0_max9_step0.50_%s" % (rx, ch, na, TAIL)))
    return out


CURVES = _curves()


def curve_name(c):
    if c["family"] == "csi1":
        tag = "eps%.2f" % c["eps"]
    elif c["family"] == "toi":
        tag = "toi%g" % c["toi"]
    elif c["family"] == "ebn0":
        tag = "ibo%g" % c["ibo"]
    elif c["family"] == "small2":
        lo, hi, st = c["ebn0_range"]
        tag = "ibo%g_ebn0_%d_%d_%g" % (c["ibo"], lo, hi, st)
    elif c["family"] == "ibo2":
        lo, hi, st = c["ibo_range"]
        tag = "ebn0_%g_ibo%d_%d_%g" % (c["ebn0"], lo, hi, st)
    else:
        tag = "eps%.1f" % c["eps"] if c["family"] == "csi" else "ebn0_%g" % c["ebn0"]
    return "%s_%s_%s_nant%d_%s" % (c["family"], c["receiver"], c["channel"], c["n_ant"], tag)


def published(c):
    import utilities
    rows = np.asarray(utilities.read_from_csv("published_" + c["file"], directory=GOLDEN), dtype=np.float64)
    return rows[0], rows[1:]  # axis; counter rows x points (ROW_MAPS)


# Published counter row -> engine column ([clean, standard RX, iterations 1..8]).  The CSI
# files hold all ten rows the committed drivers write ("full").  The BER-vs-IBO files hold
# nine, written by earlier driver revisions, in two layouts the data tell apart (the
# no-distortion row is flat in IBO and 0 at Eb/N0 1000; the standard RX falls with IBO):
# the 64-antenna LoS files are [clean, standard RX, iterations 1..7] ("prefix"); the
# Rayleigh / two-path IBO 0..8.5 files and the 1- / 4-antenna files are [standard RX,
# iterations 1..8] -- incl_clean_run False, as final_plots/ber_vs_ibo.py:22-40 reads them
# ("no_clean").  measure() reports the fit of the other layouts too.
ROW_MAPS = {"full": lambda r: list(range(r)), "prefix": lambda r: list(range(r)),
            "no_clean": lambda r: list(range(1, r + 1)), "skip_std": lambda r: [0] + list(range(2, r + 1))}


def layout(c, axis=None, pub=None):
    """Row layout of a published file.  Ten rows: [clean, standard RX, iterations 1..8].  Nine
    rows: decided by the data -- a first row that falls with IBO (Spearman rho < -0.8) is the
    standard RX ("no_clean"); a flat one is the no-distortion run ("prefix").  The rule
    reproduces every layout the fits tell apart (the wrong layouts: mean z^2 1e2-1e8)."""
    if c["family"] in ("csi", "csi1", "toi", "ebn0", "small2") or (pub is not None and pub.shape[0] == len(ITERS) + 1):
        return "full"
    if c["family"] in ("ibo", "ibo2") and pub is not None:
        from scipy.stats import spearmanr
        r0 = pub[0]
        rho = 0.0 if np.all(r0 == r0[0]) else float(spearmanr(axis, r0)[0])
        return "no_clean" if rho < -0.8 else "prefix"
    return "prefix" if c["family"] == "ibo" and c["channel"] == "los" else "no_clean"


def toi_alpha_estimate(toi_db, n_sym=10000, seed=4321, chunk=500):
    """The TOI drivers' alpha_estimate (main_miso_cnc_ber_vs_ebn0_toi.py:95-121), restated.
    The array is not precoded yet, so every antenna sends the same PA output and
    rx_k / clean_k = Y_k / X_k on every in-band bin whatever the channel: alpha = the mean over
    n_sym symbols of |mean_k Y_k / X_k|, X = the symbol's QAM points, Y = FFT(PA(IFFT(X))),
    the PA at the modem's average sample power (distortion.py:222-241)."""
    import modulation
    mod = modulation.OfdmQamModem(constel_size=M, n_fft=N_FFT, n_sub_carr=N_SC, cp_len=1)
    coeff = 1.0 / 10 ** (toi_db / 10) / mod.avg_sample_power
    k = np.arange(N_SC)
    bins = np.where(k < N_SC // 2, N_FFT - N_SC // 2 + k, k - N_SC // 2 + 1)  # modulation.py:266-267
    const = np.asarray(mod.constellation)
    rng = np.random.default_rng(seed)
    acc, done = 0.0, 0
    while done < n_sym:
        n = min(chunk, n_sym - done)
        s = const[rng.integers(0, M, (n, N_SC))]
        fd = np.zeros((n, N_FFT), complex)
        fd[:, bins] = s
        x = np.fft.ifft(fd, norm="ortho", axis=1)
        y = x - coeff * x * np.abs(x) ** 2                      # _process_toi (distortion.py:202-211)
        r = np.fft.fft(y, norm="ortho", axis=1)[:, bins] / s
        acc += float(np.abs(r.mean(axis=1)).sum())
        done += n
    return acc / n_sym


def points(c, axis):
    """Per-point engine parameters, through the Link's own object state (update_distortion /
    set_snr as the drivers call them)."""
    from link_util import build_link
    from utilities import ebn0_to_snr
    if c["family"] == "toi":
        # the geometry / channel / receiver of a Link; the PA is a point parameter (the mp Link
        # itself takes no TOI array: it reads impairment.ibo_db, mp_model.py:83)
        link, mod = build_link(n_ant=c["n_ant"], n_sc=N_SC, n_fft=N_FFT, M=M, cp=128, ibo=0.0, chan="two_path",
                               is_mcnc=c["receiver"] == "mcnc")
        alpha = toi_alpha_estimate(c["toi"])
        coeff = 1.0 / 10 ** (c["toi"] / 10) / mod.avg_sample_power  # unprecoded gain 1 (see the docstring)
        pts = []
        for v in axis:
            link.set_snr(float(ebn0_to_snr(float(v), N_SC, N_SC, M)))
            pp = link.point_params()
            pp.update(pa_kind="toi", sat_pow=0.0, toi_coeff=coeff, cnc_pa_kind="toi", cnc_sat_pow=0.0,
                      cnc_toi_coeff=coeff, cnc_alpha=alpha, array_alpha=alpha)
            pts.append(pp)
        c["alpha_estimate"] = alpha
        return link, pts
    link, _ = build_link(n_ant=c["n_ant"], n_sc=N_SC, n_fft=N_FFT, M=M, cp=128, ibo=0.0, chan=c["channel"],
                         is_mcnc=c["receiver"] == "mcnc", csi=c["eps"])
    pts = []
    for v in axis:
        ibo, ebn0 = (c["ibo"], v) if c["axis"] == "ebn0" else (v, c["ebn0"])
        link.update_distortion(float(ibo))
        link.set_snr(float(ebn0_to_snr(float(ebn0), N_SC, N_SC, M)))
        pts.append(link.point_params())
    return link, pts


def stop_trials(ber, bits_max, n_err_min):
    """Trials the reference's stopping rule gives a counter of this BER (at least one)."""
    cap = np.ceil(bits_max / BPS)
    with np.errstate(divide="ignore"):
        need = np.where(ber > 0, np.ceil(n_err_min / np.maximum(ber, 1e-300) / BPS), cap)
    return np.maximum(1.0, np.minimum(cap, need))


def run_engine(link, pts, n_tr, seed0, precision=None):
    import _engine
    from channel import carrier_freqs
    m, rx = link.my_mod, link.my_standard_rx
    eng = _engine.Engine(link.n_ant_val, m.n_sub_carr, m.n_fft, m.constel_size, m.cp_len, link._chan_kind(),
                         "mcnc" if link.is_mcnc else "cnc", link.my_array.positions(),
                         (link.rx_loc_x, link.rx_loc_y, rx.cord_z), link.rx_loc_var,
                         carrier_freqs(m.n_fft, rx.carrier_spacing, rx.center_freq), device=0, precision=precision)
    n_pt = len(pts)
    t0 = time.perf_counter()
    err, bits, per = eng.run_points(pts, [seed0 + j for j in range(n_pt)], [0] * n_pt, [n_tr] * n_pt, ITERS, True,
                                    per_trial=True)
    dt = time.perf_counter() - t0
    eng.close()
    return err, bits, per.reshape(n_pt, n_tr, len(ITERS) + 1), dt


def compare(ber, sd, q, pub, n_tr, bits_max, n_err_min, err, k_ref=1.0):
    """z statistics, bias and zero-region figures of one curve ([counter, point] arrays).
    ``k_ref`` scales the published value's variance (1: the stated stopping rule; a scatter
    factor measured from the published re-runs, tch(), otherwise)."""
    n_ref = stop_trials(ber, bits_max, n_err_min)
    sig_gpu = sd / np.sqrt(n_tr)
    sig_ref = sd * np.sqrt(k_ref / n_ref)
    ref_errs = pub * n_ref * BPS
    sel = (pub >= 1e-5) & (ref_errs >= 100) & (sd > 0)
    z = (ber - pub) / np.sqrt(sig_gpu ** 2 + sig_ref ** 2 + 1e-300)
    rel = (ber - pub) / np.where(sel, pub, 1.0)
    zs = np.abs(z[sel])
    zero = pub == 0              # the reference saw no erroneous symbol in n_ref trials
    p_zero = np.where(zero, (1.0 - q) ** n_ref, 1.0)
    ours_zero = (err == 0) & (pub > 0)
    rows = range(pub.shape[0])
    # the trial count that would make the published scatter about the engine's estimate
    # normal (mean z^2 = 1 with sigma_ref = sd / sqrt(n)): compare with the stopping rule's
    d2, sd2, sg2 = (ber - pub)[sel] ** 2, sd[sel] ** 2, sig_gpu[sel] ** 2
    n_eff = None
    if zs.size:
        lo, hi = 1.0, 1e7
        for _ in range(100):
            mid = np.sqrt(lo * hi)
            lo, hi = (mid, hi) if np.mean(d2 / (sg2 + sd2 / mid)) < 1.0 else (lo, mid)
        n_eff = round(float(np.sqrt(lo * hi)), 1)
    out = dict(compared=int(sel.sum()), n_ref_median=float(np.median(n_ref[sel])) if zs.size else None,
               n_eff=n_eff,
               frac_abs_z_le1=round(float((zs <= 1).mean()), 4) if zs.size else None,
               frac_abs_z_le2=round(float((zs <= 2).mean()), 4) if zs.size else None,
               mean_z2=round(float((zs ** 2).mean()), 3) if zs.size else None,
               max_abs_z=round(float(zs.max()), 3) if zs.size else None,
               median_abs_rel=round(float(np.median(np.abs(rel[sel]))), 5) if zs.size else None,
               row_mean_z={str(r): round(float(z[r][sel[r]].mean()), 3) for r in rows if sel[r].sum() >= 3},
               row_mean_rel={str(r): round(float(rel[r][sel[r]].mean()), 5) for r in rows if sel[r].sum() >= 3},
               zero_points=int(zero.sum()), min_p_zero=round(float(p_zero.min()), 6),
               pub_pos_ours_zero=int(ours_zero.sum()),
               pub_pos_ours_zero_max_ref_errs=round(float(ref_errs[ours_zero].max()), 2) if ours_zero.any() else 0.0)
    return out, z, sel


def measure(c, n_tr=None, seed0=5150, f32_check=False, k_ref=1.0):
    """The engine's estimate of every counter of every point of curve ``c`` against the
    published one.  Returns (summary dict, arrays)."""
    axis, pub = published(c)
    n_pt, R = len(axis), pub.shape[0]
    if n_tr is None:
        n_tr = 4096 if c["receiver"] == "mcnc" and c["n_ant"] > 4 else 8192
    link, pts = points(c, axis)
    err, bits, per, dt = run_engine(link, pts, n_tr, seed0)
    ber = (err / bits).T                                    # [column, point]
    sd = (per.astype(np.float64) / BPS).std(axis=1, ddof=1).T
    q = (per > 0).mean(axis=1).T                            # fraction of trials holding any error
    main = layout(c, axis, pub)
    maps = [main] if R == len(ITERS) + 1 else [main] + [m for m in ("prefix", "no_clean", "skip_std") if m != main]
    out = dict(curve=curve_name(c), file=c["file"], n_tr=n_tr, points=n_pt, rows=R, layout=main,
               seconds=round(dt, 2))
    if "alpha_estimate" in c:
        out["alpha_estimate"] = round(c["alpha_estimate"], 6)
    arrays = None
    for name in maps:
        cols = ROW_MAPS[name](R)
        st, z, sel = compare(ber[cols], sd[cols], q[cols], pub, n_tr, c["bits_max"], c["n_err_min"], err.T[cols],
                             k_ref)
        if name == main:
            out.update(st)
            out["z_map"] = [[round(float(v), 2) if s else None for v, s in zip(zr, sr)] for zr, sr in zip(z, sel)]
            arrays = dict(axis=axis, ber=ber[cols], pub=pub, z=z, sel=sel)
        else:
            out["alt_" + name] = dict(mean_z2=st["mean_z2"], frac_abs_z_le1=st["frac_abs_z_le1"],
                                      compared=st["compared"])
    if f32_check:
        e32, b32, per32, _ = run_engine(link, pts, n_tr, seed0, precision="f32")
        out["f32_entry_agreement"] = round(float((per32 == per).mean()), 6)
        out["f32_total_err_ratio"] = round(float(e32.sum() / max(1, err.sum())), 6)
        cols = ROW_MAPS[main](R)
        st32, _, _ = compare((e32 / b32).T[cols], sd[cols], q[cols], pub, n_tr, c["bits_max"], c["n_err_min"],
                             e32.T[cols], k_ref)
        out["f32_mean_z2"], out["f32_compared"] = st32["mean_z2"], st32["compared"]
    return out, arrays


# ---------------------------------------------------------------------------------------
# Three-cornered hat over published re-runs.  Where the reference published two independent
# runs of the same quantity -- the step-1 CSI files (csi1) re-run the 0.5-dB CSI files (csi)
# at eps 0 .. 0.4 (other Eb/N0 grids, so other seeds per point) -- the engine and the two runs
# are three independent estimates of one value.  Per point, in units of the
# engine's per-trial spread sd and of run A's stopping-rule trial count n_a (rho = n_a / n_b):
#   U = n_a ((e - a) / sd)^2 = n_a / n_tr + k_a + beta
#   V = n_a ((e - b) / sd)^2 = n_a / n_tr + k_b rho + beta
#   W = n_a ((a - b) / sd)^2 =              k_a + k_b rho
# k_a, k_b: each run's variance against its stated stopping rule's (1: the rule holds);
# beta: the engine's squared bias in units of run A's sigma^2.  Least squares over the points,
# standard errors by resampling whole points (the rows of a point share their trials).  No
# stopping-rule assumption enters beta: the two runs' own disagreement calibrates it.


def pairs():
    """The published re-run pairs (run A, run B, rows both files hold for the same quantity)."""
    by = {(c["family"], c["receiver"], c["channel"], c.get("eps"), c.get("ibo")): c for c in CURVES}
    out = []
    for rx in ("cnc", "mcnc"):
        for eps in (0.0, 0.1, 0.2, 0.3, 0.4):
            out.append(dict(name="csi1_vs_csi_%s_los_eps%.1f" % (rx, eps), a=by[("csi1", rx, "los", eps, 0.0)],
                            b=by[("csi", rx, "los", eps, 0.0)], rows=list(range(len(ITERS) + 1))))
    # Not pairs: a CNC and an MCNC file's shared rows (no-distortion, standard RX).  The drivers'
    # fixed seeds make them largely the same trials -- at IBO 1 over LoS they agree to 0.01-0.03 %,
    # far inside their binomial sigma (tests/test_published_data.py) -- so their difference does
    # not measure their scatter.
    return out


def scatter_factors(res):
    """Pooled scatter factor per (family, receiver) from tch() results: the median over the
    pairs of run A's k (csi1) and run B's k (csi)."""
    out = {}
    for rx in ("cnc", "mcnc"):
        rs = [r for r in res if r.get("pair", "").startswith("csi1_vs_csi_%s_" % rx) and "k_a" in r]
        if rs:
            out[("csi1", rx)] = float(np.median([r["k_a"] for r in rs]))
            out[("csi", rx)] = float(np.median([r["k_b"] for r in rs]))
    return out


def tch_solve(ber, sd, pa, pb, n_tr, n_a, n_b, sel, n_boot=1000, seed=0):
    """(k_a, k_b, beta) and their resampling standard errors from [row, point] arrays
    (``sel``: the cells compared; ``n_tr``: the engine's trials, a scalar or per cell)."""
    cols = np.flatnonzero(sel.any(axis=0))
    if cols.size < 4:
        return None

    nt_all = np.broadcast_to(np.asarray(n_tr, dtype=np.float64), ber.shape)  # engine trials (scalar or per cell)

    def fit(idx):
        s = sel[:, idx]
        e, d, a, b = ber[:, idx][s], sd[:, idx][s], pa[:, idx][s], pb[:, idx][s]
        na, rho = n_a[:, idx][s], (n_a / n_b)[:, idx][s]
        off = na / nt_all[:, idx][s]
        U, V, W = na * ((e - a) / d) ** 2 - off, na * ((e - b) / d) ** 2 - off, na * ((a - b) / d) ** 2
        one, zero = np.ones_like(U), np.zeros_like(U)
        X = np.concatenate([np.stack([one, zero, one], 1), np.stack([zero, rho, one], 1), np.stack([one, rho, zero], 1)])
        return np.linalg.lstsq(X, np.concatenate([U, V, W]), rcond=None)[0]

    est = fit(cols)
    rng = np.random.default_rng(seed)
    boot = np.array([fit(rng.choice(cols, cols.size)) for _ in range(n_boot)])
    se = boot.std(axis=0, ddof=1)
    return dict(k_a=round(float(est[0]), 4), k_b=round(float(est[1]), 4), beta=round(float(est[2]), 4),
                se_k_a=round(float(se[0]), 4), se_k_b=round(float(se[1]), 4), se_beta=round(float(se[2]), 4),
                points=int(cols.size), cells=int(sel.sum()))


# Files the published data alone flag as not runs of their stated configuration
# (tests/test_published_data.py): not used as a corner.
HAT_EXCLUDED = {"ibo2_cnc_los_nant64_ebn0_15_ibo0_8_0.5", "ibo_cnc_two_path_nant64_ebn0_15"}


def hat_groups(min_runs=2):
    """BER-vs-IBO files at 64 antennas that are independent runs of the same quantities: the
    same receiver, channel and Eb/N0 (driver settings 1e7 bits / 1e5 errors for all), on IBO
    grids that share points."""
    import collections
    g = collections.defaultdict(list)
    for c in CURVES:
        if c["family"] in ("ibo", "ibo2") and c["n_ant"] == 64 and curve_name(c) not in HAT_EXCLUDED:
            g[(c["receiver"], c["channel"], c["ebn0"])].append(c)
    return [dict(name="ibo_%s_%s_ebn0_%g" % k, runs=v) for k, v in sorted(g.items()) if len(v) >= min_runs]


def nch_solve(ber, sd, pubs, valid, n_rule, n_tr, same_idx, n_boot=1000, seed=0):
    """N-cornered hat: m published runs (``pubs[i]``, ``valid[i]``: [row, point]) of one rule
    (``n_rule``: its trials per cell), the engine (``ber``, ``n_tr`` trials, per-trial spread
    ``sd``).  In units of the rule's variance sd^2 / n_rule, per cell:
      U_i  = n_rule ((e - p_i) / sd)^2 - n_rule / n_tr = k_i + beta
      W_ij = n_rule ((p_i - p_j) / sd)^2               = k_i + k_j   (cells where ``same_idx[i][j]``
                                                                      is False: independent draws)
    Least squares for (k_1..k_m, beta); standard errors by resampling whole points."""
    m = len(pubs)
    P = ber.shape[1]
    cols = np.flatnonzero(np.any([v.any(axis=0) for v in valid], axis=0))
    nt_all = np.broadcast_to(np.asarray(n_tr, dtype=np.float64), ber.shape)

    def fit(idx):
        X, y = [], []
        for i in range(m):
            s = valid[i][:, idx]
            n = n_rule[:, idx][s]
            u = n * ((ber[:, idx][s] - pubs[i][:, idx][s]) / sd[:, idx][s]) ** 2 - n / nt_all[:, idx][s]
            row = np.zeros(m + 1)
            row[i], row[m] = 1.0, 1.0
            X.append(np.tile(row, (u.size, 1)))
            y.append(u)
            for j in range(i + 1, m):
                s2 = valid[i][:, idx] & valid[j][:, idx] & ~same_idx[i][j][:, idx]
                n = n_rule[:, idx][s2]
                w = n * ((pubs[i][:, idx][s2] - pubs[j][:, idx][s2]) / sd[:, idx][s2]) ** 2
                row = np.zeros(m + 1)
                row[i], row[j] = 1.0, 1.0
                X.append(np.tile(row, (w.size, 1)))
                y.append(w)
        return np.linalg.lstsq(np.concatenate(X), np.concatenate(y), rcond=None)[0]

    est = fit(cols)
    rng = np.random.default_rng(seed)
    boot = np.array([fit(rng.choice(cols, cols.size)) for _ in range(n_boot)])
    se = boot.std(axis=0, ddof=1)
    pairs = sum(int((valid[i] & valid[j] & ~same_idx[i][j]).sum()) for i in range(m) for j in range(i + 1, m))
    return dict(k=[round(float(x), 4) for x in est[:m]], se_k=[round(float(x), 4) for x in se[:m]],
                beta=round(float(est[m]), 4), se_beta=round(float(se[m]), 4), points=int(cols.size),
                cells=int(sum(v.sum() for v in valid)), pair_cells=pairs)


def nch(grp, n_tr=None, seed0=5150):
    """The engine on the union of a hat group's IBO points; nch_solve over its runs (the counter
    rows every run's layout holds)."""
    runs = grp["runs"]
    pubs_raw = [published(c) for c in runs]
    axis = np.unique(np.round(np.concatenate([a for a, _ in pubs_raw]), 6))
    c0 = runs[0]
    if n_tr is None:
        n_tr = 4096 if c0["receiver"] == "mcnc" else 8192
    link, pts = points(c0, axis)
    err, bits, per, dt = run_engine(link, pts, n_tr, seed0)
    ber_all = (err / bits).T                                            # [engine column, point]
    sd_all = (per.astype(np.float64) / BPS).std(axis=1, ddof=1).T
    maps = [ROW_MAPS[layout(c, a, p)](p.shape[0]) for c, (a, p) in zip(runs, pubs_raw)]
    common = sorted(set.intersection(*[set(mp) for mp in maps]))
    ber, sd = ber_all[common], sd_all[common]
    R, P = len(common), axis.size
    pubs, valid, gidx = [], [], []
    n_rule = stop_trials(ber, c0["bits_max"], c0["n_err_min"])
    for c, (a, p), mp in zip(runs, pubs_raw, maps):
        full = np.full((R, P), np.nan)
        gi = np.full(P, -1)
        for j, x in enumerate(axis):
            hit = np.flatnonzero(np.isclose(a, x))
            if hit.size:
                full[:, j] = p[[mp.index(col) for col in common], hit[0]]
                gi[j] = hit[0]
        ok = np.isfinite(full) & (full >= 1e-5) & (np.nan_to_num(full) * n_rule * BPS >= 100) & (sd > 0)
        pubs.append(np.nan_to_num(full))
        valid.append(ok)
        gidx.append(gi)
    m = len(runs)
    same = [[np.broadcast_to((gidx[i] == gidx[j]) & (gidx[i] >= 0), (R, P)) for j in range(m)] for i in range(m)]
    res = nch_solve(ber, sd, pubs, valid, n_rule, n_tr, same)
    res.update(group=grp["name"], runs=[curve_name(c) for c in runs], rows=R, n_tr=n_tr, seconds=round(dt, 2),
               n_rule_median=float(np.median(n_rule[np.any(valid, axis=0)])) if any(v.any() for v in valid) else None)
    res["bias_rms_2se"] = round(float(np.sqrt(max(0.0, res["beta"] + 2 * res["se_beta"]))), 4)
    return res


def tch(p, n_tr=None, seed0=5150):
    """The engine at the common points of a published pair; tch_solve's figures, plus each run's
    effective trial count (its rule's median over k)."""
    ca, cb = p["a"], p["b"]
    axa, puba = published(ca)
    axb, pubb = published(cb)
    common = np.array([x for x in axa if np.any(np.isclose(axb, x))])
    ia = [int(np.flatnonzero(np.isclose(axa, x))[0]) for x in common]
    ib = [int(np.flatnonzero(np.isclose(axb, x))[0]) for x in common]
    if n_tr is None:
        n_tr = 4096 if ca["receiver"] == "mcnc" else 8192
    link, pts = points(ca, common)
    err, bits, per, dt = run_engine(link, pts, n_tr, seed0)
    rows = p["rows"]
    cols_a = ROW_MAPS[layout(ca, axa, puba)](puba.shape[0])
    ber = (err / bits).T[cols_a][rows]
    sd = (per.astype(np.float64) / BPS).std(axis=1, ddof=1).T[cols_a][rows]
    pa, pb = puba[rows][:, ia], pubb[rows][:, ib]
    n_a = stop_trials(ber, ca["bits_max"], ca["n_err_min"])
    n_b = stop_trials(ber, cb["bits_max"], cb["n_err_min"])
    sel = (pa >= 1e-5) & (pb >= 1e-5) & (pa * n_a * BPS >= 100) & (pb * n_b * BPS >= 100) & (sd > 0)
    # a point with the same grid index in both files may share its seeds (the 0.5-dB CSI eps-0
    # and IBO-0 LoS files, one grid, agree to 0.2 % against ~1 % for independent runs): not used
    sel[:, np.asarray(ia) == np.asarray(ib)] = False
    out = dict(pair=p["name"], a=ca["file"], b=cb["file"], n_tr=n_tr, points=len(common), rows=len(rows),
               seconds=round(dt, 2))
    res = tch_solve(ber, sd, pa, pb, n_tr, n_a, n_b, sel)
    if res is not None:
        out.update(res)
        out["n_rule_a"], out["n_rule_b"] = float(np.median(n_a[sel])), float(np.median(n_b[sel]))
        out["n_eff_a"] = round(out["n_rule_a"] / max(res["k_a"], 1e-9), 1)
        out["n_eff_b"] = round(out["n_rule_b"] / max(res["k_b"], 1e-9), 1)
        # the bias the engine may still have at 2 standard errors, in units of run A's sigma
        out["bias_rms_2se"] = round(float(np.sqrt(max(0.0, res["beta"] + 2 * res["se_beta"]))), 4)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--family", default="all")
    ap.add_argument("--out", default=None)
    ap.add_argument("--n-tr", type=int, default=None)
    ap.add_argument("--pairs", action="store_true", help="the three-cornered hat over the published re-run pairs")
    ap.add_argument("--hat", action="store_true", help="the N-cornered hat over the BER-vs-IBO re-run groups")
    a = ap.parse_args()
    if a.hat:
        res = []
        for g in hat_groups():
            r = nch(g, a.n_tr)
            print(json.dumps(r), flush=True)
            res.append(r)
        if a.out:
            with open(a.out, "w") as f:
                json.dump(res, f, indent=1)
        return
    if a.pairs:
        res = []
        for p in pairs():
            r = tch(p, a.n_tr)
            print(json.dumps(r), flush=True)
            res.append(r)
        # each family's scatter factor, pooled per receiver over the paired eps 0 .. 0.4 runs,
        # applied to every curve of that family (the unpaired csi1 curves are the same driver
        # revision's runs)
        ks = scatter_factors(res)
        for c in CURVES:
            k = ks.get((c["family"], c["receiver"]))
            if k is not None:
                r, _ = measure(c, a.n_tr, k_ref=k)
                r = {kk: v for kk, v in r.items() if kk != "z_map"}
                r["k_ref"] = round(k, 4)
                print(json.dumps(r), flush=True)
                res.append(r)
        if a.out:
            with open(a.out, "w") as f:
                json.dump(res, f, indent=1)
        return
    res = []
    for c in CURVES:
        if a.family != "all" and c["family"] != a.family:
            continue
        r, _ = measure(c, a.n_tr, f32_check=c.get("ebn0") == 1000.0)
        print(json.dumps(r), flush=True)
        res.append(r)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
