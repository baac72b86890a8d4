"""Per-trial Monte-Carlo BER chain on the CPU (NumPy float64) -- the engine's oracle.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg use it, as the checker / CPU baseline.

One trial = one OFDM symbol of ``Link.simulate`` (mp_model.py:180-222, and the clean run
mp_model.py:133-175) with the reference's PCG64 draws replaced by the Philox streams
of ``oracle.philox``:

* bits -> QAM labels                                   mp_model.py:208
* channel reroll (Rayleigh / LoS / two-path)           mp_model.py:190-204, channel.py
* (CSI error) + MRT precoding + AGC                    mp_model.py:253-329, antenna_array.py:162-185
* per-antenna OFDM TX + PA, FFT                        antenna_array.py:127-132, transceiver.py:155-159
* channel combine, AWGN, AGC divide                    mp_model.py:210-214, channel.py:287-290, noise.py:56-83
* CNC / MCNC receiver, bit-error count                 corrector.py:52-112 / 165-207, mp_model.py:215-222

Counters per trial: ``[clean?] + [one per entry of iters]`` (mp_model.py:127-131,217-222).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import philox
from . import refmath as rm


@dataclass
class SimConfig:
    n_ant: int
    n_sc: int
    n_fft: int
    constel_size: int
    pa: str = "softlim"            # softlim | rapp | toi | none
    p_hardness: float = 3.0
    ibo_db: float = 3.0
    snr_db: float = 20.0           # value passed to Link.set_snr (already Eb/N0 -> SNR)
    channel: str = "rayleigh"      # rayleigh | los | two_path | table (fixed matrix table_h)
    receiver: str = "cnc"          # cnc | mcnc
    csi_eps: float | None = None
    center_freq: float = 3.5e9
    carrier_spacing: float = 15e3
    array_z: float = 15.0
    wav_len_spacing: float = 0.5
    rx_pos: tuple = (212.0, 212.0, 1.5)
    rx_loc_var: float = 10.0
    reroll: bool = True
    tx_pos: np.ndarray | None = field(default=None, repr=False)
    table_h: np.ndarray | None = field(default=None, repr=False)  # [A, F] channel_mat_fd for "table"
    csi_seed: int | None = None    # "table" + CSI: key of the one shared estimate (None: the run seed)
    # the TOI drivers' measured alpha_estimate (main_miso_cnc_ber_vs_ebn0_toi.py:95-134,247-249):
    # every antenna's AGC gain and the CNC receiver's alpha; None: Link's (mp_model.py:315-317)
    array_alpha: float | None = None
    cnc_alpha: float | None = None

    def __post_init__(self):
        if self.tx_pos is None:
            self.tx_pos = rm.ula_positions(self.n_ant, self.center_freq, self.wav_len_spacing, self.array_z)


def _const(cfg):
    return rm.gray_qam_constellation(cfg.constel_size)


def channel_inband(cfg: SimConfig, z_chan, loc_u):
    """True in-band channel [A, S] for one trial."""
    bins = rm.inband_bins(cfg.n_fft, cfg.n_sc)
    if cfg.channel == "table":
        # Link.simulate(reroll_chan=False): the channel object's matrix for every trial
        return np.asarray(cfg.table_h, dtype=np.complex128)[:, bins]
    if cfg.channel == "rayleigh":
        # MisoRayleighFd.reroll_channel_coeffs (channel.py:262-275): CN(0,1) x FSPL at the
        # nominal RX position (the Rayleigh RX does not move, mp_model.py:191).
        att = rm.fspl_matrix(cfg.tx_pos, cfg.rx_pos, cfg.n_fft, cfg.carrier_spacing, cfg.center_freq)
        return z_chan * att[:, bins]
    # LoS / two-path: RX moved by U(-var/2, var/2) in x and y, both around rx_loc_x
    # (mp_model.py:192-199 uses rx_loc_x for the y coordinate too).
    x0 = cfg.rx_pos[0]
    if cfg.reroll:
        rx = (x0 - cfg.rx_loc_var / 2 + cfg.rx_loc_var * loc_u[0],
              x0 - cfg.rx_loc_var / 2 + cfg.rx_loc_var * loc_u[1], cfg.rx_pos[2])
    else:
        rx = cfg.rx_pos
    fn = rm.los_channel if cfg.channel == "los" else rm.two_path_channel
    return fn(cfg.tx_pos, rx, cfg.n_fft, cfg.carrier_spacing, cfg.center_freq)[:, bins]


def point_params(cfg: SimConfig):
    """Per-grid-point scalars that ``Link`` keeps in its objects."""
    const = _const(cfg)
    es = rm.avg_symbol_power(const)
    avg_samp = es * cfg.n_sc / cfg.n_fft
    out = dict(const=const, es=es, avg_samp=avg_samp, snr=10 ** (cfg.snr_db / 10))
    if cfg.pa == "toi":
        out["cnc_coeff"] = rm.toi_coeff(cfg.ibo_db, avg_samp)
        out["cnc_alpha"] = 1.0
        out["cnc_sat"] = 0.0
    else:
        # CncReceiver: sat = 10^(IBO/10) * Es * S/F, alpha = calc_alpha(IBO)
        # (corrector.py:23-50 + Link.update_distortion, mp_model.py:230-241).
        out["cnc_sat"] = rm.sat_pow(cfg.ibo_db, avg_samp)
        out["cnc_alpha"] = float(rm.calc_alpha(cfg.ibo_db))
        out["cnc_coeff"] = 0.0
    if cfg.cnc_alpha is not None:
        out["cnc_alpha"] = float(cfg.cnc_alpha)
    return out


def _tx_pa(cfg, x_sc, pp, gain):
    """Per-antenna OFDM TX with PA, back to the in-band FD: [A, S] -> [A, S]."""
    bins = rm.inband_bins(cfg.n_fft, cfg.n_sc)
    fd = np.zeros((x_sc.shape[0], cfg.n_fft), dtype=np.complex128)
    fd[:, bins] = x_sc
    td = np.fft.ifft(fd, norm="ortho", axis=-1)
    avg = pp["avg_samp"] * gain  # AntennaArray.update_distortion (antenna_array.py:337-360)
    if cfg.pa == "toi":
        td = rm.toi(rm.toi_coeff(cfg.ibo_db, avg), td)
    elif cfg.pa != "none":
        td = rm.apply_pa(cfg.pa, td, rm.sat_pow(cfg.ibo_db, avg), cfg.p_hardness)
    return np.fft.fft(td, norm="ortho", axis=-1)[:, bins]


def run_trial(cfg: SimConfig, labels, z_chan, z_noise, loc_u=None, z_csi=None, iters=(0,),
              incl_clean=False, return_debug=False):
    """One trial; returns error counts [clean?] + [per iteration in ``iters``]."""
    pp = point_params(cfg)
    const = pp["const"]
    nb = rm.bits_per_symbol(cfg.constel_size)
    s = const[labels]
    h = channel_inband(cfg, z_chan, loc_u)
    h_est = rm.csi_error(h, cfg.csi_eps, z_csi) if cfg.csi_eps is not None else h
    p = rm.mrt_precoding(h_est)
    gain = rm.avg_precoding_gain(p)
    g = rm.agc(h_est, p, cfg.ibo_db, cfg.n_sc, cfg.n_ant, cfg.array_alpha)
    counts = []

    def nerr(lab):
        return int(np.bitwise_count(np.asarray(lab, np.int64) ^ labels).sum()) if hasattr(np, "bitwise_count") \
            else int(rm.labels_to_bits(np.asarray(lab) ^ labels, nb).sum())

    if incl_clean:
        # clean run: no PA; IFFT->FFT round trip is the identity in-band (mp_model.py:159-169)
        r_c = np.sum(h * (s[None, :] * p), axis=0)
        n_c = np.sqrt(pp["es"] * g["hk_vk_noise"] / pp["snr"]) * z_noise
        z_c = (r_c + n_c) / g["hk_vk"]
        counts.append(nerr(rm.detect_labels(const, z_c)))

    y = _tx_pa(cfg, s[None, :] * p, pp, gain)
    r = np.sum(h * y, axis=0)
    n = np.sqrt(pp["es"] * g["ak_hk_vk_noise"] / pp["snr"]) * z_noise
    z = (r + n) / g["ak_hk_vk"]
    iters = [int(i) for i in iters]
    if cfg.receiver == "cnc":
        det = rm.cnc_receive(iters, z, const, cfg.n_fft, cfg.pa, pp["cnc_sat"], cfg.p_hardness,
                             pp["cnc_coeff"], pp["cnc_alpha"])
    else:
        det = mcnc_receive(cfg, iters, z, const, p, h_est, g["ak_hk_vk"], pp, gain)
    counts.extend(nerr(det[i]) for i in iters)
    if return_debug:
        return counts, dict(z=z, h=h, p=p, agc=g, gain=gain)
    return counts


def mcnc_receive(cfg, iters, z, const, p, h_prop, agc_vec, pp, gain):
    """``McncReceiver.receive`` (corrector.py:165-207): re-transmit detected symbols
    through the whole array + PA + (estimated) channel every iteration."""
    out = {}
    d = None
    for it in range(max(iters) + 1):
        v = z if it == 0 else z - d
        lab = rm.detect_labels(const, v)
        s_hat = const[lab]
        if it in iters:
            out[it] = lab
        y = _tx_pa(cfg, s_hat[None, :] * p, pp, gain)
        est = np.sum(h_prop * y, axis=0) / agc_vec
        d = est - s_hat
    return out


FIXED_CSI_TRIAL = 0xFFFFFFFF  # CSI stream counter of fixed-channel runs (csrc/trial_kernel.h kFixedCsiTrial)


def draws(cfg: SimConfig, seed: int, trials):
    """All random inputs of a batch of trials from the Philox streams."""
    trials = np.asarray(trials, dtype=np.int64)
    out = dict(labels=philox.qam_labels(seed, trials, cfg.n_sc, cfg.constel_size),
               z_chan=philox.chan_normals(seed, trials, cfg.n_sc, cfg.n_ant),
               z_noise=philox.noise_normals(seed, trials, cfg.n_sc),
               loc_u=philox.loc_uniforms(seed, trials))
    if cfg.csi_eps is not None:
        # a fixed channel (reroll_chan=False) keeps the one erroneous estimate Link.__init__
        # drew (mp_model.py:87; set_precoding_and_recalculate_agc is not called in the loop,
        # :190-206): every trial reads the same, trial-independent CSI draw
        # and, as the estimate belongs to the Link, from the Link's own key (csi_seed), not the run's
        fixed = cfg.channel == "table"
        csi_trials = np.full_like(trials, FIXED_CSI_TRIAL) if fixed else trials
        csi_key = cfg.csi_seed if fixed and cfg.csi_seed else seed
        out["z_csi"] = philox.csi_normals(csi_key, csi_trials, cfg.n_sc, cfg.n_ant)
    return out


def run_trials(cfg: SimConfig, seed: int, trials, iters=(0,), incl_clean=False, chunk=8):
    """Error counts [n_trials, n_idx] for the given trial ids."""
    trials = np.asarray(trials, dtype=np.int64)
    rows = []
    for i in range(0, len(trials), chunk):
        d = draws(cfg, seed, trials[i:i + chunk])
        for j in range(len(trials[i:i + chunk])):
            rows.append(run_trial(cfg, d["labels"][j], d["z_chan"][j], d["z_noise"][j], d["loc_u"][j],
                                  d["z_csi"][j] if "z_csi" in d else None, iters, incl_clean))
    return np.asarray(rows, dtype=np.int64)
