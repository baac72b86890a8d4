"""How much the reference's channel replay widens the scatter of its published BER curves.

The reference's drivers fork W = num_cores workers per grid point, and every worker
deep-copies the same seeded Rayleigh generator (channel.py:209-212, mp_model.py:61): the
W workers replay ONE channel sequence, with their own bits and noise.  A published BER is
therefore an average over N trials (its stopping rule) that hold only ceil(N / W) distinct
channels, and its variance is larger than N independent trials give.

This tool emulates that estimator on the GPU (mimo_config.chan_replay_period = ceil(N / W):
trial i draws the channel of trial i mod period) R times per point with different seeds,
takes the spread of those R estimates as the published value's sigma, and compares the
engine's own estimate (independent channels, n_tr trials) with the published curves of the
paper config (CSV data files of figs/csv_results in tests/golden) by
z = (ber - pub) / sqrt(sigma_gpu^2 + sigma_ref(W)^2), for several W.

    python tools/replay_sigma.py [--out file.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "m-mimo-ofdm-with-nonlinear-pa-sim_amd"), os.path.join(REPO, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

CURVES = [("cnc", "rayleigh"), ("mcnc", "rayleigh"), ("cnc", "los"), ("mcnc", "los"), ("cnc", "two_path"),
          ("mcnc", "two_path")]
ITERS = [0, 1, 2, 3, 4]
BPS = 2048 * 6
BITS_MAX, N_ERR_MIN = 1e7, 1e6  # main_mp_miso_cnc_ber_vs_ebn0.py:57-58


def published(receiver, channel):
    import utilities
    d = os.path.join(REPO, "tests", "golden")
    name = ("published_ber_vs_ebn0_cnc_rayleigh_ibo3" if (receiver, channel) == ("cnc", "rayleigh") else
            "published_ber_vs_ebn0_%s_%s_nant64_ibo3_ebn0_min5_max20_step1.00_niter1_2_3_4_5_6_7_8" % (receiver, channel))
    rows = np.asarray(utilities.read_from_csv(name, directory=d))
    return rows[0], rows[1:2 + len(ITERS)]  # axis; no-distortion (clean), standard RX, iterations 1..4


def engine(receiver, channel, period):
    from gpu_util import engine_for
    from oracle import sim
    cfg = sim.SimConfig(64, 2048, 4096, 64, pa="softlim", ibo_db=3.0, snr_db=20.0, channel=channel, receiver=receiver)
    import _engine
    from oracle import refmath as rm
    carriers = rm.fftfreq_carriers(cfg.n_fft, cfg.carrier_spacing, cfg.center_freq)
    eng = _engine.Engine(cfg.n_ant, cfg.n_sc, cfg.n_fft, cfg.constel_size, 4, cfg.channel, cfg.receiver, cfg.tx_pos,
                         cfg.rx_pos, cfg.rx_loc_var, carriers, device=-1, chan_replay_period=int(period))
    return eng, engine_for


def point_kw(ebn0):
    from oracle import sim
    c = sim.SimConfig(64, 2048, 4096, 64, pa="softlim", ibo_db=3.0, snr_db=float(sim.rm.ebn0_to_snr(ebn0, 2048, 2048, 64)))
    pp = sim.point_params(c)
    return dict(ibo_db=c.ibo_db, snr_db=c.snr_db, avg_symbol_power=pp["es"], pa_kind="softlim",
                sat_pow=sim.rm.sat_pow(c.ibo_db, pp["avg_samp"] / c.n_ant), cnc_pa_kind="softlim",
                cnc_sat_pow=pp["cnc_sat"], cnc_alpha=pp["cnc_alpha"])


def measure(receiver, channel, workers=(1, 4, 8, 16, 32), reps=24, n_tr=8192):
    ebn0, pub = published(receiver, channel)
    n_pt = len(ebn0)
    pts = [point_kw(e) for e in ebn0]
    # the engine's own estimate: independent channels, n_tr trials per point, batch-means sigma
    eng, _ = engine(receiver, channel, 0)
    err, bits, per = eng.run_points(pts, [4242 + j for j in range(n_pt)], [0] * n_pt, [n_tr] * n_pt, ITERS, True,
                                    per_trial=True)
    ber = (err / bits).T
    per = per.reshape(n_pt, n_tr, len(ITERS) + 1).astype(np.float64) / BPS
    sig_gpu = per.std(axis=1, ddof=1).T / np.sqrt(n_tr)
    # the reference's trial count per point (all counters share trials; a counter closes at
    # n_err_min errors or the bit budget)
    n_ref = np.minimum(BITS_MAX / BPS, np.ceil(N_ERR_MIN / np.maximum(pub, 1e-300) / BPS).max(axis=0)).astype(int)
    sel = pub >= 1e-4
    # bias view (independent of sigma): relative difference per compared point, its median
    # magnitude, and its mean per counter row (rows with >= 3 compared points)
    rel = (ber - pub) / np.where(sel, pub, 1.0)
    row_bias = {str(r): round(float(rel[r][sel[r]].mean()), 5) for r in range(len(pub)) if sel[r].sum() >= 3}
    out = dict(receiver=receiver, channel=channel, n_tr=n_tr, reps=reps, n_ref=n_ref.tolist(), compared=int(sel.sum()),
               median_abs_rel=round(float(np.median(np.abs(rel[sel]))), 5), row_mean_rel=row_bias, by_workers={})
    for W in workers:
        sig_ref = np.zeros_like(pub)
        engines = {}
        for j in range(n_pt):
            period = int(np.ceil(n_ref[j] / W))
            if period not in engines:
                engines[period] = engine(receiver, channel, period if W > 1 else 0)[0]
            e_r, b_r, _ = engines[period].run_points([pts[j]] * reps, [777000 + 1000 * j + r for r in range(reps)],
                                                     [0] * reps, [int(n_ref[j])] * reps, ITERS, True)
            est = e_r / b_r  # [reps, idx]
            sig_ref[:, j] = est.std(axis=0, ddof=1)
        for e in engines.values():
            e.close()
        z = (ber - pub) / np.sqrt(sig_gpu ** 2 + sig_ref ** 2 + 1e-300)
        zs = np.abs(z[sel])
        out["by_workers"][str(W)] = dict(frac_abs_z_le1=round(float((zs <= 1).mean()), 4),
                                         frac_abs_z_le2=round(float((zs <= 2).mean()), 4),
                                         mean_z2=round(float((zs ** 2).mean()), 3), max_abs_z=round(float(zs.max()), 3),
                                         median_sigma_ref_over_gpu=round(float(np.median((sig_ref / sig_gpu)[sel])), 3))
    return out, dict(ber=ber, pub=pub, sig_gpu=sig_gpu)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--reps", type=int, default=24)
    a = ap.parse_args()
    res = []
    for rx, ch in CURVES:
        # only the Rayleigh generator is replayed: LoS / two-path reroll the RX position from
        # the per-worker reseeded loc_rng (mp_model.py:121-125,190-201), independent per worker
        r, _ = measure(rx, ch, workers=(1, 4, 8, 16, 32) if ch == "rayleigh" else (1,), reps=a.reps)
        print(json.dumps(r), flush=True)
        res.append(r)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
