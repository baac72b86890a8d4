"""Capture golden vectors by running the REFERENCE (read-only at /root/reference).

Run in the build container only:  ``python tests/golden/make_golden.py``.
The reference never travels; only the ``*.npz`` fixtures written next to this file do.

Import recipe: two ``sys.modules`` stubs -- ``numba`` (``objmode`` is a
no-op context outside jitted code, ``jit`` the identity, as ``speedup.py:2-19`` already
falls back to) and an empty ``matlab.engine`` (only QuaDRiGa / LDPC would touch it).

Two kinds of fixtures:

* ``units.npz``  -- deterministic library calls on recorded inputs: constellations, hard
  demod incl. lattice tie points, LLRs, alpha(IBO), soft limiter / Rapp / TOI, OFDM TX/RX,
  MRT precoding + PA calibration + AGC on a recorded channel, array transmit, CNC and MCNC
  receivers on a recorded received vector.
* ``link_<name>.npz`` -- end-to-end ``mp_model.Link.simulate`` runs in which the
  reference's PCG64 generators are replaced by stubs that serve the engine's Philox
  draws (``oracle.philox``) in the reference's own call order.  Each trial is one
  ``simulate`` call (clean trial + distorted trial), so the fixture holds the
  reference's per-trial, per-iteration bit-error counts for Philox-addressed inputs that
  the oracle and the GPU engine regenerate from the stored seed.
"""
from __future__ import annotations

import contextlib
import ctypes
import multiprocessing as mp
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)


def import_reference():
    import matplotlib
    matplotlib.use("Agg")
    numba = types.ModuleType("numba")
    numba.objmode = lambda **kw: contextlib.nullcontext()
    numba.jit = lambda *a, **k: (a[0] if a and callable(a[0]) else (lambda f: f))
    sys.modules["numba"] = numba
    matlab = types.ModuleType("matlab")
    eng = types.ModuleType("matlab.engine")
    matlab.engine = eng
    sys.modules["matlab"] = matlab
    sys.modules["matlab.engine"] = eng
    sys.path.insert(0, REF)
    import modulation, distortion, channel, noise, transceiver, antenna_array, corrector, utilities, mp_model  # noqa
    return types.SimpleNamespace(modulation=modulation, distortion=distortion, channel=channel, noise=noise,
                                 transceiver=transceiver, antenna_array=antenna_array, corrector=corrector,
                                 utilities=utilities, mp_model=mp_model)


R = import_reference()
from oracle import philox  # noqa: E402
from oracle import refmath as rm  # noqa: E402

FC, DF = int(3.5e9), int(15e3)


# ----------------------------------------------------------------------------- system builder
def build_system(n_ant, n_sc, n_fft, M, cp, pa="softlim", ibo=3.0, p_hard=3.0, chan="rayleigh"):
    mod = R.modulation.OfdmQamModem(constel_size=M, n_fft=n_fft, n_sub_carr=n_sc, cp_len=cp)
    if pa == "softlim":
        dist = R.distortion.SoftLimiter(0, mod.avg_sample_power)
    elif pa == "rapp":
        dist = R.distortion.Rapp(ibo_db=0, p_hardness=p_hard, avg_samp_pow=mod.avg_sample_power)
    else:
        raise ValueError(pa)
    import copy
    tx = R.transceiver.Transceiver(modem=copy.deepcopy(mod), impairment=copy.deepcopy(dist), center_freq=FC,
                                   carrier_spacing=DF)
    rx = R.transceiver.Transceiver(modem=copy.deepcopy(mod), impairment=copy.deepcopy(dist), cord_x=212.0,
                                   cord_y=212.0, cord_z=1.5, center_freq=FC, carrier_spacing=DF)
    arr = R.antenna_array.LinearArray(n_elements=n_ant, base_transceiver=tx, center_freq=FC, wav_len_spacing=0.5,
                                      cord_x=0, cord_y=0, cord_z=15)
    if chan == "rayleigh":
        ch = R.channel.MisoRayleighFd(tx_transceivers=arr.array_elements, rx_transceiver=rx, seed=1234)
    elif chan == "los":
        ch = R.channel.MisoLosFd()
        ch.calc_channel_mat(tx_transceivers=arr.array_elements, rx_transceiver=rx, skip_attenuation=False)
    elif chan == "two_path":
        ch = R.channel.MisoTwoPathFd()
        ch.calc_channel_mat(tx_transceivers=arr.array_elements, rx_transceiver=rx, skip_attenuation=False)
    noise = R.noise.Awgn(snr_db=10, seed=1234)
    return mod, dist, tx, rx, arr, ch, noise


# ----------------------------------------------------------------------------- RNG stubs
class Feed:
    """Serves recorded draws in the reference's call order, checking each request."""

    def __init__(self):
        self.q = []

    def push(self, kind, value):
        self.q.append((kind, value))

    def _pop(self, kind):
        if not self.q:
            raise RuntimeError(f"feed exhausted, wanted {kind}")
        k, v = self.q.pop(0)
        if k != kind:
            raise RuntimeError(f"feed order: wanted {kind}, next is {k}")
        return v

    def standard_normal(self, size=None):
        v = self._pop(("normal", tuple(size)))
        return v.copy()

    def choice(self, a, size):
        return self._pop(("choice", int(size))).copy()

    def uniform(self, low=0.0, high=1.0):
        u = self._pop(("uniform",))
        return low + (high - low) * u


def push_trial(feeds, sys_cfg, d, j, csi):
    """Queue the draws of one trial in Link.simulate's consumption order."""
    A, S, F, M, chan = sys_cfg
    bins = rm.inband_bins(F, S)
    nb = rm.bits_per_symbol(M)
    if chan == "rayleigh":
        zf = np.zeros((A, F), complex)
        zf[:, bins] = d["z_chan"][j]
        n = np.empty((A, 2 * F))
        n[:, 0::2] = np.sqrt(2) * zf.real
        n[:, 1::2] = np.sqrt(2) * zf.imag
        feeds["chan"].push(("normal", (A, 2 * F)), n)
    else:
        feeds["loc"].push(("uniform",), float(d["loc_u"][j][0]))
        feeds["loc"].push(("uniform",), float(d["loc_u"][j][1]))
    if csi:
        for a in range(A):
            zc = d["z_csi"][j][a]
            feeds["noise"].push(("normal", (S, 2)), np.stack([np.sqrt(2) * zc.real, np.sqrt(2) * zc.imag], axis=1))
    feeds["bits"].push(("choice", S * nb), rm.labels_to_bits(d["labels"][j], nb).astype(np.int64))
    zn = np.zeros(F, complex)
    zn[bins] = d["z_noise"][j]
    feeds["noise"].push(("normal", (F, 2)), np.stack([np.sqrt(2) * zn.real, np.sqrt(2) * zn.imag], axis=1))


def run_link(name, n_ant, n_sc, n_fft, M, cp, pa, ibo, p_hard, chan, ebn0, iters, n_trials, seed,
             mcnc=False, csi=None, incl_clean=True):
    mod, dist, tx, rx, arr, ch, noise = build_system(n_ant, n_sc, n_fft, M, cp, pa, ibo, p_hard, chan)
    link = R.mp_model.Link(mod_obj=mod, array_obj=arr, std_rx_obj=rx, chan_obj=ch, noise_obj=noise,
                           rx_loc_var=10.0, n_err_min=10 ** 12, bits_sent_max=mod.n_bits_per_ofdm_sym,
                           is_mcnc=mcnc, csi_epsylon=csi)
    link.update_distortion(ibo_val_db=ibo)
    snr_db = float(R.utilities.ebn0_to_snr(ebn0, mod.n_sub_carr, mod.n_sub_carr, mod.constel_size))
    link.set_snr(snr_db_val=snr_db)
    iters = np.asarray(iters)
    feeds = {k: Feed() for k in ("chan", "bits", "noise", "loc", "csi")}
    link.my_miso_chan.rng_gen = feeds["chan"]
    rng_by_seed = {11: feeds["bits"], 12: feeds["noise"], 13: feeds["loc"], 14: feeds["csi"]}

    cfg_sim_kw = dict(n_ant=n_ant, n_sc=n_sc, n_fft=n_fft, constel_size=M, pa=pa, p_hardness=p_hard, ibo_db=ibo,
                      snr_db=snr_db, channel=chan, receiver="mcnc" if mcnc else "cnc", csi_eps=csi)
    from oracle.sim import SimConfig, draws
    cfg = SimConfig(**cfg_sim_kw)
    trials = np.arange(n_trials)
    d = draws(cfg, seed, trials)
    sys_cfg = (n_ant, n_sc, n_fft, M, chan)

    captured = {}
    orig_receive = link.my_cnc_rx.receive

    def spy(n_iters_lst, in_sig_fd, *a, **k):
        captured.setdefault("z", []).append(np.asarray(in_sig_fd).copy())
        return orig_receive(n_iters_lst, in_sig_fd, *a, **k)

    link.my_cnc_rx.receive = spy
    orig_default_rng = np.random.default_rng
    counts = []
    try:
        np.random.default_rng = lambda s=None: rng_by_seed[int(s)]
        for j in range(n_trials):
            for _ in range(2 if incl_clean else 1):
                push_trial(feeds, sys_cfg, d, j, csi is not None)
            n_idx = len(iters) + (1 if incl_clean else 0)
            err = mp.Array(ctypes.c_double, n_idx, lock=True)
            bits = mp.Array(ctypes.c_double, n_idx, lock=True)
            link.simulate(incl_clean, True, iters, [11, 12, 13, 14], err, bits)
            counts.append(np.asarray(err[:], dtype=np.int64))
            assert all(b == mod.n_bits_per_ofdm_sym for b in bits[:]), bits[:]
            for f in feeds.values():
                assert not f.q, "unconsumed draws"
    finally:
        np.random.default_rng = orig_default_rng
    counts = np.asarray(counts)
    z_bins = rm.inband_bins(n_fft, n_sc)
    z0 = np.asarray(captured["z"][0])[z_bins]
    out = dict(counts=counts, seed=np.int64(seed), n_trials=np.int64(n_trials), iters=iters,
               incl_clean=np.int64(incl_clean), snr_db=np.float64(snr_db), ebn0=np.float64(ebn0),
               n_ant=np.int64(n_ant), n_sc=np.int64(n_sc), n_fft=np.int64(n_fft), M=np.int64(M), cp=np.int64(cp),
               pa=np.array(pa), ibo=np.float64(ibo), p_hard=np.float64(p_hard), chan=np.array(chan),
               mcnc=np.int64(mcnc), csi=np.float64(-1.0 if csi is None else csi), z_trial0=z0,
               labels_sum=np.int64(d["labels"].sum()), zchan_abs_sum=np.float64(np.abs(d["z_chan"]).sum()))
    np.savez_compressed(os.path.join(HERE, f"link_{name}.npz"), **out)
    print(name, "BER per index:", counts.sum(0) / (n_trials * mod.n_bits_per_ofdm_sym))


# ----------------------------------------------------------------------------- unit fixtures
def make_units():
    rng = np.random.default_rng(20240607)
    out = {}
    for M in (4, 16, 64, 256):
        m = R.modulation.QamModem(M)
        out[f"const_{M}"] = np.asarray(m.constellation)
        L = int(np.sqrt(M))
        # random points + lattice boundary (tie) points
        pts = (rng.uniform(-L - 1, L + 1, 600) + 1j * rng.uniform(-L - 1, L + 1, 600))
        grid = np.arange(-L, L + 1, 1.0)
        gi, gq = np.meshgrid(grid, grid)
        ties = (gi + 1j * gq).reshape(-1)
        halfties = (np.round(rng.uniform(-L, L, 200)) + 1j * rng.uniform(-L, L, 200))
        allp = np.concatenate([pts, ties, halfties, halfties.imag + 1j * halfties.real])
        out[f"demod_in_{M}"] = allp
        out[f"demod_bits_{M}"] = np.asarray(R.modulation.demodulate(m.constellation, m.n_bits_per_symbol, allp))
        out[f"symdet_{M}"] = np.asarray(m.symbol_detection(allp))
        bits = rng.integers(0, 2, 60 * m.n_bits_per_symbol)
        out[f"mod_bits_{M}"] = bits
        out[f"mod_out_{M}"] = np.asarray(R.modulation.modulate(m.constellation, m.n_bits_per_symbol, bits))
    # LLR (soft decoding) on 16-QAM
    m16 = R.modulation.OfdmQamModem(16, 128, 64, 4)
    z = (rng.normal(size=64) + 1j * rng.normal(size=64)) * 2
    out["llr_in"] = z
    out["llr_out"] = np.asarray(m16.soft_detection_llr(z, 0.7))
    # alpha
    ibo = np.arange(-5, 15.01, 0.25)
    out["alpha_ibo"] = ibo
    out["alpha_out"] = np.asarray(m16.calc_alpha(ibo))
    # PA models
    x = (rng.normal(size=500) + 1j * rng.normal(size=500)) * 4
    x[:5] = [0, 1 + 1j, 3 + 4j, 10, -20j]
    out["pa_in"] = x
    sl = R.distortion.SoftLimiter(3, 20.95)
    out["pa_softlim_sat"] = np.float64(sl.sat_pow)
    out["pa_softlim_out"] = sl.process(x)
    for p in (3, 4, 5):
        ra = R.distortion.Rapp(3, 20.95, p)
        out[f"pa_rapp{p}_out"] = ra.process(x)
    toi = R.distortion.ThirdOrderNonLin(12, 20.95)
    out["pa_toi_coeff"] = np.float64(toi.cubic_dist_coeff)
    out["pa_toi_out"] = toi.process(x)
    # OFDM TX / RX
    for (F, S, cp) in ((128, 64, 4), (2048, 1024, 128)):
        mod = R.modulation.OfdmQamModem(64, F, S, cp)
        bits = rng.integers(0, 2, mod.n_bits_per_ofdm_sym)
        out[f"ofdm_bits_{F}"] = bits
        td = mod.modulate(bits)
        out[f"ofdm_td_{F}"] = td
        out[f"ofdm_rxsym_{F}"] = mod.demodulate(td, get_symbols_only=True)
        out[f"ofdm_rxbits_{F}"] = np.asarray(mod.demodulate(td))
    # array-level: precoding, PA calibration, AGC, transmit, CNC, MCNC on a recorded channel
    A, S, F, M, cp = 4, 64, 128, 16, 4
    mod, dist, tx, rx, arr, ch, noise = build_system(A, S, F, M, cp, "softlim", 2.0, 3.0, "rayleigh")
    link = R.mp_model.Link(mod_obj=mod, array_obj=arr, std_rx_obj=rx, chan_obj=ch, noise_obj=noise, rx_loc_var=10.0,
                           n_err_min=10, bits_sent_max=10, is_mcnc=False)
    link.update_distortion(ibo_val_db=2.0)
    h = np.asarray(link.my_miso_chan.channel_mat_fd)
    out["arr_H"] = h
    out["arr_P"] = np.asarray(link.my_array.get_precoding_mat())
    out["arr_sat"] = np.asarray([e.impairment.sat_pow for e in link.my_array.array_elements])
    out["arr_ak_agc"] = np.asarray(link.ak_hk_vk_agc_nfft)
    out["arr_hk_agc"] = np.asarray(link.hk_vk_agc_nfft)
    out["arr_ak_noise"] = np.float64(link.ak_hk_vk_noise_scaler)
    out["arr_hk_noise"] = np.float64(link.hk_vk_noise_scaler)
    bits = rng.integers(0, 2, mod.n_bits_per_ofdm_sym)
    out["arr_bits"] = bits
    out["arr_tx_fd"] = np.asarray(link.my_array.transmit(bits, out_domain_fd=True, skip_dist=False))
    out["arr_tx_fd_clean"] = np.asarray(link.my_array.transmit(bits, out_domain_fd=True, skip_dist=True))
    r = link.my_miso_chan.propagate(in_sig_mat=out["arr_tx_fd"])
    r = r + 0.05 * (rng.normal(size=F) + 1j * rng.normal(size=F))
    r = r / link.ak_hk_vk_agc_nfft
    out["cnc_in"] = r
    out["cnc_sat"] = np.float64(link.my_cnc_rx.impairment.sat_pow)
    out["cnc_alpha"] = np.float64(link.my_cnc_rx.modem.alpha)
    res = link.my_cnc_rx.receive(n_iters_lst=np.array([0, 1, 2, 3, 5]), in_sig_fd=r)
    out["cnc_iters"] = np.array([0, 1, 2, 3, 5])
    out["cnc_bits"] = np.stack([np.asarray(b) for b in res])
    mlink = R.mp_model.Link(mod_obj=mod, array_obj=arr, std_rx_obj=rx, chan_obj=ch, noise_obj=noise, rx_loc_var=10.0,
                            n_err_min=10, bits_sent_max=10, is_mcnc=True)
    mlink.update_distortion(ibo_val_db=2.0)
    mlink.my_miso_chan.channel_mat_fd = h
    mlink.my_cnc_rx.channel = mlink.my_miso_chan
    mlink.set_precoding_and_recalculate_agc()
    resm = mlink.my_cnc_rx.receive(n_iters_lst=np.array([0, 1, 2, 3]), in_sig_fd=r)
    out["mcnc_iters"] = np.array([0, 1, 2, 3])
    out["mcnc_bits"] = np.stack([np.asarray(b) for b in resm])
    # geometry / channels
    out["ula_x"] = np.asarray([e.cord_x for e in arr.array_elements])
    los = R.channel.MisoLosFd()
    los.calc_channel_mat(tx_transceivers=arr.array_elements, rx_transceiver=rx)
    out["los_H"] = np.asarray(los.channel_mat_fd)
    tp = R.channel.MisoTwoPathFd()
    tp.calc_channel_mat(tx_transceivers=arr.array_elements, rx_transceiver=rx)
    out["twopath_H"] = np.asarray(tp.channel_mat_fd)
    out["rayleigh_att"] = np.asarray(ch.los_fd_att_mat)
    out["ebn0_to_snr"] = np.asarray(R.utilities.ebn0_to_snr(np.arange(0, 31.0), 1024, 1024, 64))
    np.savez_compressed(os.path.join(HERE, "units.npz"), **out)
    print("units.npz:", len(out), "arrays")


if __name__ == "__main__":
    make_units()
    # name, A, S, F, M, cp, pa, ibo, p, chan, ebn0, iters, trials, seed, [mcnc, csi]
    run_link("small_cnc", 4, 64, 128, 16, 4, "softlim", 0.0, 3.0, "rayleigh", 10.0, [0, 1, 2, 3], 40, 1234)
    run_link("mid_cnc", 16, 256, 512, 64, 16, "softlim", 3.0, 3.0, "rayleigh", 15.0, [0, 1, 2, 3, 4], 24, 2137)
    run_link("cfg2_cnc", 64, 1024, 2048, 64, 128, "softlim", 3.0, 3.0, "rayleigh", 15.0, [0, 1, 2, 3, 4], 8, 2137)
    run_link("rapp", 8, 128, 256, 16, 8, "rapp", 2.0, 3.0, "rayleigh", 12.0, [0, 1, 2], 24, 77)
    # a CNC run (no mcnc=True): written as link_small_mcnc.npz, renamed link_a8_cnc.npz in round 6
    # (file name only; the data are as captured).  No Link-level capture has is_mcnc=True: MCNC
    # is pinned by the reference at the receiver level (units.npz mcnc_bits, make_units above).
    run_link("a8_cnc", 8, 64, 128, 16, 4, "softlim", 1.0, 3.0, "rayleigh", 12.0, [0, 1, 2], 16, 99)
    run_link("los_cnc", 8, 128, 256, 64, 8, "softlim", 3.0, 3.0, "los", 20.0, [0, 1, 2], 16, 5)
    run_link("twopath_cnc", 8, 128, 256, 64, 8, "softlim", 3.0, 3.0, "two_path", 20.0, [0, 1, 2], 16, 6)
    run_link("csi_cnc", 8, 128, 256, 16, 8, "softlim", 2.0, 3.0, "rayleigh", 12.0, [0, 1, 2], 16, 7, csi=0.3)
    print("done")
