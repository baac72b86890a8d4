"""Test-side helpers: build a GPU Engine for an oracle SimConfig (same system, same point)."""
import numpy as np

from oracle import refmath as rm
from oracle.sim import SimConfig, point_params


PRECISIONS = ["f64", "f32"]  # every parity test runs both instances of the fused kernel


def engine_for(cfg: SimConfig, device=-1, precision=None):
    import _engine
    carriers = rm.fftfreq_carriers(cfg.n_fft, cfg.carrier_spacing, cfg.center_freq)
    eng = _engine.Engine(cfg.n_ant, cfg.n_sc, cfg.n_fft, cfg.constel_size, 4, cfg.channel, cfg.receiver, cfg.tx_pos,
                         cfg.rx_pos, cfg.rx_loc_var, carriers, reroll=cfg.reroll, device=device, precision=precision,
                         chan_table=cfg.table_h if cfg.channel == "table" else None,
                         csi_seed=cfg.csi_seed or 0)
    pp = point_params(cfg)
    avg = pp["avg_samp"] / cfg.n_ant  # MRT: mean |P|^2 = 1/A (antenna_array.py:328-335)
    if cfg.pa == "toi":
        kw = dict(toi_coeff=rm.toi_coeff(cfg.ibo_db, avg))
    else:
        kw = dict(sat_pow=rm.sat_pow(cfg.ibo_db, avg))
    eng.point_kw = dict(ibo_db=cfg.ibo_db, snr_db=cfg.snr_db, avg_symbol_power=pp["es"], pa_kind=cfg.pa,
                        p_hardness=cfg.p_hardness, cnc_pa_kind=cfg.pa, cnc_sat_pow=pp["cnc_sat"],
                        cnc_toi_coeff=pp["cnc_coeff"], cnc_alpha=pp["cnc_alpha"], csi_eps=cfg.csi_eps, array_alpha=cfg.array_alpha, **kw)
    eng.set_point(**eng.point_kw)
    return eng


def assert_counts_equal(per, ref, label=""):
    """Per-trial, per-iteration bit-error counts must agree EXACTLY (both kernels, both
    precisions: the device sees the oracle's Philox draws, so only a received point
    within rounding distance of a slicer boundary could flip; none does on these cases)."""
    per = np.asarray(per, np.int64)
    ref = np.asarray(ref, np.int64)
    assert per.shape == ref.shape, (per.shape, ref.shape)
    bad = np.argwhere(per != ref)
    assert bad.size == 0, f"{label}: {len(bad)} of {per.size} entries differ, first {bad[:5].tolist()}"


def count_agreement(a, b):
    """Fraction of (trial, index) entries that agree exactly."""
    a = np.asarray(a, np.int64)
    b = np.asarray(b, np.int64)
    return float(np.mean(a == b))
