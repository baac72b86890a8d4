"""BASELINE config 4 on the GPU against the reference's published fixed-BER grids.

Runs ``sweep.run_grid`` exactly as the reference's fixed-BER driver sets up its grid
(main_mp_miso_cnc_constant_ber_req_ebn0_vs_ibo.py:100-215: 64-antenna ULA, N_fft 4096,
2048 sub-carriers, 64-QAM, soft limiter, IBO 0..7.5 dB x Eb/N0 10..22 dB in 0.5 dB steps,
receiver iterations 0..8, no clean run, bits_sent_max 5e6, n_err_min 1e5) and compares
every (IBO, Eb/N0, iteration) BER with the published CSV
(tests/golden/published_fixed_ber1.0e-02_<rx>_<channel>_nant64_...csv, a data file of the
reference's figs/csv_results) by a z-score.

sigma: replicas of the reference's estimator.  Every point is re-run ``reps`` times with
independent seeds at the trial count the reference's stopping rule gave it (from the
published BERs: all counters share trials; a counter closes at n_err_min errors or the bit
budget); the spread of those estimates is the published value's sigma, and the GPU
estimate's sigma is the same spread scaled by sqrt(reference trials / trials run).  (The
reference's workers replay one Rayleigh sequence, channel.py:209-212; tools/replay_sigma.py
measured that replay to change these sigmas by < 5 % at 64 antennas, so the replicas draw
independent channels.)

    python tools/fixed_ber_check.py --channel rayleigh --receiver cnc [--precision f64]
    python tools/fixed_ber_check.py --grid baseline      # BASELINE config 4 at its stated extent

``--grid baseline`` runs BASELINE.json's config 4 extent (SNR 0-30 dB x IBO 0-7 dB; SURVEY
§8(d) C4: Eb/N0 0..30 dB in 0.5 dB steps x IBO 0..7 dB in 0.5 dB steps = 915 points, CNC
0..8, bits_sent_max 5e6, n_err_min 1e5, paper geometry) on one GPU and times it.  There is
no published grid at that extent, so it is a throughput / coverage run with property
checks instead of a comparison: every counter of every point closed by the stopping rule,
BER non-increasing in Eb/N0 for the standard receiver at every IBO (beyond sampling noise),
and the 400 points it shares with the published grid agree with it (z-scores).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "m-mimo-ofdm-with-nonlinear-pa-sim_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

GOLDEN = os.path.join(REPO, "tests", "golden")
IBO = np.arange(0.0, 8.0, 0.5)
EBN0 = np.arange(10.0, 22.1, 0.5)
ITERS = np.arange(0, 9)
N_ANT, N_SC, N_FFT, M, CP = 64, 2048, 4096, 64, 128
BITS_MAX, N_ERR_MIN = int(5e6), int(1e5)


def published(channel, receiver, n_ant=N_ANT, ibo_step=0.5):
    """The published grid: IBO 0..7 in ``ibo_step`` steps (0.5 for the four paper grids; the
    0.25-step 64-antenna and the 1-antenna files are other runs of the same driver)."""
    import utilities
    name = ("published_fixed_ber1.0e-02_%s_%s_nant%d_ebn0_min10_max22_step0.50_ibo_min0_max7_step%.2f_"
            "niter1_2_3_4_5_6_7_8" % (receiver, channel, n_ant, ibo_step))
    rows = utilities.read_from_csv(name, directory=GOLDEN)
    ibo = np.asarray(rows[0], dtype=np.float64)
    ber = np.asarray(rows[1:], dtype=np.float64).reshape(len(ibo), -1, len(ITERS))
    return ibo, ber


def build_link(channel, receiver, precision, n_ant=N_ANT):
    import sweep
    return sweep.paper_link(channel, receiver, precision, n_ant=n_ant, n_sc=N_SC, n_fft=N_FFT, qam=M, cp=CP,
                            n_err_min=N_ERR_MIN, bits_sent_max=BITS_MAX)


def reference_trials(pub_ber, bits_per_sym, per_counter=False):
    """Trials the reference's stopping rule needed per point: every counter closes at
    n_err_min errors or at the bit budget (it stops accumulating then, mp_model.py:181-187,
    217-222); the point stops when all are closed.  per_counter: each counter's own count."""
    budget = BITS_MAX / bits_per_sym
    need = np.where(pub_ber > 0, N_ERR_MIN / np.maximum(pub_ber, 1e-300) / bits_per_sym, budget)
    if per_counter:
        return np.minimum(budget, np.ceil(need))
    return np.minimum(budget, np.ceil(need.max(axis=-1)))


def run(channel="rayleigh", receiver="cnc", precision="f64", reps=16, seed=2137, n_ant=N_ANT, ibo_step=0.5,
        detail=None):
    """The engine's grid against one published grid (module docstring).  ``detail`` (a dict,
    optional) receives the per-cell arrays the comparison used: the replica sigma, the
    reference's and the engine's trial counts per counter."""
    import sweep
    from utilities import ebn0_to_snr
    IBO = np.arange(0.0, 8.0, ibo_step)  # noqa: N806 (the grid of this published file)
    link = build_link(channel, receiver, precision, n_ant)
    bits_per_sym = N_SC * int(np.log2(M))
    link.engine().run(0, 0, 1, [0])  # engine / device set-up and code-object load outside the timed sweep
    t0 = time.perf_counter()
    err, bits = sweep.run_grid(link, IBO, EBN0, ITERS, incl_clean=False, seed=seed)
    wall = time.perf_counter() - t0
    # a point's trials: its counters share them, and the one open longest saw them all (iteration
    # 0 closes first in a fixed-BER grid), so the largest counter, not counter 0
    trials = bits.max(axis=-1) / bits_per_sym
    trials_c = bits / bits_per_sym            # per counter: a closed counter stops accumulating
    ber = err / bits
    # replicas of the reference's estimator at its trial counts (independent seeds)
    eng = link.engine()
    params = []
    for i in IBO:
        link.update_distortion(float(i))
        for e in EBN0:
            link.set_snr(float(ebn0_to_snr(e, N_SC, N_SC, M)))
            params.append(dict(link.point_params()))
    P = len(params)
    from mp_model import _seed64
    pub_ibo, pub = published(channel, receiver, n_ant, ibo_step)
    assert np.allclose(pub_ibo, IBO) and pub.shape == ber.shape, (pub_ibo, pub.shape, ber.shape)
    n_ref = reference_trials(pub, bits_per_sym).astype(np.int64)          # [ibo, ebn0]
    seeds = [_seed64(sweep.point_seed(seed + 1 + r, p)) for r in range(reps) for p in range(P)]
    e_r, b_r, _ = eng.run_points(params * reps, seeds, [0] * (P * reps), list(n_ref.reshape(-1)) * reps,
                                 [int(x) for x in ITERS], False)
    est = (e_r / b_r).reshape(reps, len(IBO), len(EBN0), len(ITERS))
    sig_rep = est.std(axis=0, ddof=1)         # one estimate over the point's n_ref trials
    sig_rep = np.maximum(sig_rep, np.sqrt(np.maximum(pub, 1e-12) / (bits_per_sym * n_ref[..., None])))  # floor
    # variance ~ 1 / trials: each published counter holds its own trial count, as does ours
    n_ref_c = reference_trials(pub, bits_per_sym, per_counter=True)
    sig = sig_rep * np.sqrt(n_ref[..., None] / n_ref_c + n_ref[..., None] / trials_c)
    # self-consistency of the replica sigma: the last replica against the mean of the others
    # (same trial counts, same sigma model) -- a normal sample puts ~95 % within 2 sigma
    s_loo = est[:-1].std(axis=0, ddof=1)
    z_self = (est[-1] - est[:-1].mean(axis=0)) / np.maximum(s_loo * np.sqrt(1.0 + 1.0 / (reps - 1)), 1e-300)
    if detail is not None:
        detail.update(sig_rep=sig_rep, n_ref=n_ref, n_ref_c=n_ref_c, trials_c=trials_c, ibo=IBO)
    sel = pub >= 1e-3
    z = np.where(sel, (ber - pub) / sig, 0.0)
    rel = np.where(sel, np.abs(ber - pub) / np.maximum(pub, 1e-300), 0.0)
    worst = np.unravel_index(np.argmax(np.abs(z)), z.shape)
    bias = [float(((ber - pub) / np.where(sel, pub, 1.0))[..., i][sel[..., i]].mean()) for i in range(len(ITERS))]
    req_gpu = sweep.required_ebn0(ber, EBN0, 1e-2)
    req_pub = sweep.required_ebn0(pub, EBN0, 1e-2)
    fin = np.isfinite(req_gpu) & np.isfinite(req_pub)
    dreq = np.abs(req_gpu[fin] - req_pub[fin])  # only where both are finite (no inf - inf)
    n_sym = int(trials.sum())
    spread = spread_stats(z, sel, pub)
    out = dict(channel=channel, receiver=receiver, precision=precision, n_ant=n_ant, ibo_step=ibo_step, points=int(P), ofdm_symbols=n_sym,
               wall_s=round(wall, 3), symbols_per_s=round(n_sym / wall, 1), compared=int(sel.sum()),
               max_abs_z=round(float(np.abs(z).max()), 3), p95_abs_z=round(float(np.percentile(np.abs(z[sel]), 95)), 3),
               mean_z2=round(float((z[sel] ** 2).mean()), 3),
               max_abs_bias_per_iteration=round(float(np.max(np.abs(bias))), 5),
               frac_abs_z_gt3=round(float((np.abs(z[sel]) > 3).mean()), 5),
               frac_abs_z_le1=round(float((np.abs(z[sel]) <= 1).mean()), 4),
               frac_abs_z_le2=round(float((np.abs(z[sel]) <= 2).mean()), 4),
               replica_self_check=dict(frac_abs_z_le1=round(float((np.abs(z_self[sel]) <= 1).mean()), 4),
                                       frac_abs_z_le2=round(float((np.abs(z_self[sel]) <= 2).mean()), 4)),
               median_rel=round(float(np.median(rel[sel])), 5), max_rel=round(float(rel[sel].max()), 4),
               worst=dict(ibo=float(IBO[worst[0]]), ebn0=float(EBN0[worst[1]]), iteration=int(worst[2]),
                          ber=float(ber[worst]), published=float(pub[worst]), z=float(z[worst])),
               trials_per_point=dict(min=int(trials.min()), max=int(trials.max())),
               req_ebn0_at_ber_1e2=dict(finite_mismatch=int((np.isfinite(req_gpu) != np.isfinite(req_pub)).sum()),
                                     compared=int(fin.sum()),
                                     mean_abs_db=round(float(dreq.mean()), 4) if dreq.size else None,
                                     max_abs_db=round(float(dreq.max()), 4) if dreq.size else None),
               spread=spread)
    return out, ber, pub, z


def pair_check(channel, precision="f64", reps=16, seed=2137):
    """Three-cornered hat (tools/published_families.py tch_solve) over the two published CNC
    runs of one channel's grid: the 0.5-dB paper grid (run A) and the 0.25-dB grid (run B) at
    the IBO values they share.  Per-trial spread from the replicas; each run's trials per counter
    from its stopping rule; cells with published BER >= 1e-3 in both runs.  The IBO 0 row is
    left out: it has the same grid index in both files, and over LoS the two runs agree there
    to 0.12 % against ~1 % at every other IBO (the drivers' per-point seeds coincide)."""
    import published_families as pf
    det = {}
    out, ber, pub_a, _ = run(channel, "cnc", precision, reps, seed, detail=det)
    ibo_b, pub_b_all = published(channel, "cnc", N_ANT, 0.25)
    ib = [int(np.flatnonzero(np.isclose(ibo_b, x))[0]) for x in det["ibo"]]
    pub_b = pub_b_all[ib]
    bits_per_sym = N_SC * int(np.log2(M))
    n_a = det["n_ref_c"]
    n_b = reference_trials(pub_b, bits_per_sym, per_counter=True)
    sd = det["sig_rep"] * np.sqrt(det["n_ref"][..., None])      # per-trial spread
    sel = (pub_a >= 1e-3) & (pub_b >= 1e-3) & (sd > 0)
    sel[0] = False                                               # IBO 0: shared seeds
    # [iteration, point] for tch_solve (the 9 counters of a point share its trials: resample points)
    tr = lambda x: np.moveaxis(np.asarray(x, dtype=np.float64), -1, 0).reshape(len(ITERS), -1)  # noqa: E731
    res = pf.tch_solve(tr(ber), tr(sd), tr(pub_a), tr(pub_b), tr(det["trials_c"]), tr(n_a), tr(n_b),
                       np.moveaxis(sel, -1, 0).reshape(len(ITERS), -1))
    res.update(channel=channel, precision=precision, grid_mean_z2=out["mean_z2"],
               n_rule_a=float(np.median(n_a[sel])), n_rule_b=float(np.median(n_b[sel])))
    res["bias_rms_2se"] = round(float(np.sqrt(max(0.0, res["beta"] + 2 * res["se_beta"]))), 4)
    return res


def spread_stats(z, sel, pub=None):
    """Where the excess spread of z sits.  z: [ibo, ebn0, iteration],
    sel: compared entries.

    The 9 iteration counters of a point share its trials (ours and the reference's), so
    their z are nearly one variable: ``within_point_corr`` (z of iterations i, i+1 at the
    same point) is reported, and the row / lag statistics use the POINT z (mean over the
    point's compared iterations).  Reported:
    * per iteration column: mean z over points (a calibration or physics mismatch of one
      receiver iteration shows here; bound 3 / sqrt(n) for n independent points);
    * per IBO row: mean point z, bounded by 3 sqrt(v / n) with v the measured variance of
      the point z (a signed mismatch confined to an IBO region shows here);
    * lag-1 autocorrelation of the point z along Eb/N0 within each IBO row: estimates whose
      points share randomness (the reference replaying one seeded channel sequence at
      every point, channel.py:209-212, mp_model.py:61) give positive values, independent
      per-point errors ~0 (bound 3 / sqrt(pairs));
    * the point-z variance (1 if the sigma model holds), split by stopping-rule regime
      (budget-limited: every counter below BER 2e-2 closes at bits_sent_max) and by IBO."""
    n_ibo, n_ebn0, n_it = z.shape
    pz = np.full((n_ibo, n_ebn0), np.nan)
    for i in range(n_ibo):
        for j in range(n_ebn0):
            if sel[i, j].sum() >= 1:
                pz[i, j] = z[i, j][sel[i, j]].mean()
    ok = np.isfinite(pz)
    v = float(np.nanvar(pz))
    a, b = [], []
    for i in range(n_ibo):
        for it in range(n_it - 1):
            m = sel[i, :, it] & sel[i, :, it + 1]
            a += list(z[i, m, it])
            b += list(z[i, m, it + 1])
    wcorr = float(np.corrcoef(a, b)[0, 1]) if len(a) > 2 else float("nan")
    cols = []
    for it in range(n_it):
        zz = z[..., it][sel[..., it]]
        if zz.size:
            m = float(zz.mean())
            cols.append(dict(iteration=it, n=int(zz.size), mean_z=round(m, 3), mean_z2=round(float((zz ** 2).mean()), 3),
                             bound=round(3 / np.sqrt(zz.size), 3), outside=bool(abs(m) > 3 / np.sqrt(zz.size))))
    rows = []
    for i in range(n_ibo):
        zz = pz[i][ok[i]]
        if zz.size:
            m, bd = float(zz.mean()), 3 * np.sqrt(v / zz.size)
            rows.append(dict(ibo_index=i, n_points=int(zz.size), mean_point_z=round(m, 3), bound=round(float(bd), 3),
                             outside=bool(abs(m) > bd)))
    num = d0 = d1 = 0.0
    pairs = 0
    for i in range(n_ibo):
        m = ok[i, 1:] & ok[i, :-1]
        x, y = pz[i, :-1][m], pz[i, 1:][m]
        num += float((x * y).sum())
        d0 += float((x * x).sum())
        d1 += float((y * y).sum())
        pairs += int(m.sum())
    lag1 = num / np.sqrt(d0 * d1) if d0 > 0 and d1 > 0 else float("nan")
    out = dict(within_point_corr=round(wcorr, 3), n_points=int(ok.sum()), point_z_var=round(v, 3),
               iterations=cols, rows=rows, lag1_point_z_along_ebn0=round(float(lag1), 4), lag1_pairs=pairs,
               lag1_bound=round(3 / np.sqrt(max(pairs, 1)), 4),
               iterations_outside=sum(c["outside"] for c in cols), rows_outside=sum(r["outside"] for r in rows))
    if pub is not None:
        budget = np.array([[sel[i, j].any() and pub[i, j][sel[i, j]].max() < 2e-2 for j in range(n_ebn0)]
                           for i in range(n_ibo)]) & ok
        half = np.zeros_like(ok)
        half[: n_ibo // 2 - 2] = True
        out["point_z_var_by_regime"] = dict(
            budget_limited=dict(n=int(budget.sum()), var=round(float(np.var(pz[budget])), 3) if budget.any() else None),
            error_limited=dict(n=int((ok & ~budget).sum()), var=round(float(np.var(pz[ok & ~budget])), 3)),
            ibo_below_3db=dict(n=int((ok & half).sum()), var=round(float(np.var(pz[ok & half])), 3)),
            ibo_from_3db=dict(n=int((ok & ~half).sum()), var=round(float(np.var(pz[ok & ~half])), 3)))
    return out


BASE_IBO = np.arange(0.0, 7.01, 0.5)    # 15 points (sweep.BASELINE_C4)
BASE_EBN0 = np.arange(0.0, 30.01, 0.5)  # 61 points


def run_baseline(channel="rayleigh", receiver="cnc", precision="f64", seed=2137):
    """BASELINE config 4 at its stated extent (module docstring): timed sweep + property checks."""
    import sweep
    link = build_link(channel, receiver, precision)
    bits_per_sym = N_SC * int(np.log2(M))
    link.engine().run(0, 0, 1, [0])  # engine / device set-up outside the timed sweep
    t0 = time.perf_counter()
    err, bits = sweep.run_grid(link, BASE_IBO, BASE_EBN0, ITERS, incl_clean=False, seed=seed)
    wall = time.perf_counter() - t0
    ber = err / bits
    trials = bits.max(axis=-1) / bits_per_sym  # a point's trials (its longest-open counter)
    closed = (err >= N_ERR_MIN) | (bits >= BITS_MAX)
    # standard receiver (iteration 0): BER(Eb/N0) non-increasing per IBO, beyond 4 sigma of
    # binomial noise at the measured counts (bits within a symbol are correlated: x 8 margin)
    b0 = ber[..., 0]
    sig = np.sqrt(np.maximum(b0, 1e-12) * 8.0 / bits[..., 0])
    rises = (b0[:, 1:] - b0[:, :-1]) > 4 * np.hypot(sig[:, 1:], sig[:, :-1])
    # the sub-grid shared with the published grid (IBO 0..7, Eb/N0 10..22)
    pub_ibo, pub = published(channel, receiver)
    ii = [int(np.argmin(np.abs(BASE_IBO - v))) for v in pub_ibo if v <= BASE_IBO[-1] + 1e-9]
    jj = [int(np.argmin(np.abs(BASE_EBN0 - v))) for v in EBN0]
    sub, pubs = ber[np.ix_(ii, jj)], pub[:len(ii)]
    ntr_sub = (bits / bits_per_sym)[np.ix_(ii, jj)]          # per counter
    n_ref = reference_trials(pubs, bits_per_sym, per_counter=True)
    sig_sub = np.sqrt(np.maximum(pubs, 1e-12) * 8.0 / bits_per_sym) * np.sqrt(1 / ntr_sub + 1 / n_ref)
    sel = pubs >= 1e-3
    zsub = (sub - pubs) / sig_sub
    req = sweep.required_ebn0(ber, BASE_EBN0, 1e-2)
    n_sym = int(trials.sum())
    out = dict(grid="baseline", channel=channel, receiver=receiver, precision=precision,
               points=int(len(BASE_IBO) * len(BASE_EBN0)), ibo=[float(BASE_IBO[0]), float(BASE_IBO[-1])],
               ebn0=[float(BASE_EBN0[0]), float(BASE_EBN0[-1])], iterations=[int(ITERS[0]), int(ITERS[-1])],
               ofdm_symbols=n_sym, wall_s=round(wall, 3), symbols_per_s=round(n_sym / wall, 1),
               trials_per_point=dict(min=int(trials.min()), max=int(trials.max())),
               all_counters_closed=bool(closed.all()), standard_rx_ber_rises=int(rises.sum()),
               shared_with_published=dict(points=int(len(ii) * len(jj)), compared=int(sel.sum()),
                                          median_rel=round(float(np.median(np.abs(sub - pubs)[sel] / pubs[sel])), 5),
                                          frac_abs_z_le2_binomial_x8=round(float((np.abs(zsub[sel]) <= 2).mean()), 4)),
               req_ebn0_at_ber_1e2_finite=int(np.isfinite(req).sum()))
    return out, ber


def main_pairs(precision="f64"):
    for ch in ("rayleigh", "los", "two_path"):
        print(json.dumps(pair_check(ch, precision)), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--channel", default="rayleigh", choices=["rayleigh", "los", "two_path"])
    ap.add_argument("--receiver", default="cnc", choices=["cnc", "mcnc"])
    ap.add_argument("--precision", default="f64", choices=["f64", "f32"])
    ap.add_argument("--out", default=None)
    ap.add_argument("--grid", default="published", choices=["published", "baseline", "pairs"])
    ap.add_argument("--n-ant", type=int, default=N_ANT)
    ap.add_argument("--ibo-step", type=float, default=0.5)
    a = ap.parse_args()
    if a.grid == "pairs":  # three-cornered hat over the 0.5- and 0.25-dB published CNC grids
        main_pairs(a.precision)
        return
    if a.grid == "baseline":
        out, ber = run_baseline(a.channel, a.receiver, a.precision)
        print(json.dumps(out), flush=True)
        if a.out:
            np.savez(a.out, ber=ber)
        return
    out, ber, pub, z = run(a.channel, a.receiver, a.precision, n_ant=a.n_ant, ibo_step=a.ibo_step)
    print(json.dumps(out), flush=True)
    if a.out:
        np.savez(a.out, ber=ber, pub=pub, z=z)


if __name__ == "__main__":
    main()
