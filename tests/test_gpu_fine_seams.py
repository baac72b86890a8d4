"""GPU parity of the object-API fine seams (float64 stage kernels via the C ABI) against
the reference's own outputs (tests/golden/units.npz).  Labels / bits bit-exact (incl.
lattice tie points); float arrays to 1e-9 relative (FFT ordering)."""
import copy

import numpy as np
import pytest

from link_util import build_link

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M", [4, 16, 64, 256])
def test_qam_map_demap_bit_exact(units, M):
    import modulation
    m = modulation.QamModem(M)
    np.testing.assert_array_equal(m.constellation, units[f"const_{M}"])
    np.testing.assert_array_equal(m.modulate(units[f"mod_bits_{M}"]), units[f"mod_out_{M}"])
    z = units[f"demod_in_{M}"]
    np.testing.assert_array_equal(m.demodulate(z), units[f"demod_bits_{M}"])
    np.testing.assert_array_equal(m.symbol_detection(z), units[f"symdet_{M}"])


def test_demap_scaled_constellation(units):
    """correct_constellation (alpha-scaled constellation, modulation.py:148-158) stays exact
    off the decision boundaries.  (Exact lattice ties only exist for the unscaled
    constellation: after scaling by alpha the reference's tie-break is decided by float64
    rounding of hypot, so tie points are tested unscaled above.)"""
    import modulation
    m = modulation.QamModem(16)
    m.correct_constellation(1.5)
    rng = np.random.default_rng(5)
    z = (rng.uniform(-5, 5, 4000) + 1j * rng.uniform(-5, 5, 4000)) * m.alpha
    from oracle import refmath as rm
    np.testing.assert_array_equal(m.demodulate(z), rm.demodulate(m.constellation, z))


def test_llr(units):
    import modulation
    m = modulation.OfdmQamModem(16, 128, 64, 4)
    np.testing.assert_allclose(m.soft_detection_llr(units["llr_in"], 0.7), units["llr_out"], rtol=1e-9, atol=1e-12)


def test_pa_models(units):
    import distortion
    x = units["pa_in"]
    sl = distortion.SoftLimiter(3, 20.95)
    np.testing.assert_allclose(sl.process(x), units["pa_softlim_out"], rtol=1e-12, atol=1e-14)
    for p in (3, 4, 5):
        np.testing.assert_allclose(distortion.Rapp(3, 20.95, p).process(x), units[f"pa_rapp{p}_out"], rtol=1e-12)
    np.testing.assert_allclose(distortion.ThirdOrderNonLin(12, 20.95).process(x), units["pa_toi_out"], rtol=1e-12)


def test_calc_alpha_vs_published_measured_gains():
    """The reference's measured per-antenna Bussgang gains (figs/csv_results/
    alpha_vs_tx_power_per_ant64_ibo0.0.csv, main_misc_evals/main_alpha_vs_tx_pow_per_ant_eval.py:
    64 antennas under MRT at IBO 0, 1e4 symbols, rows (per-antenna IBO, measured alpha) for
    Rayleigh, two-path and LoS): the engine's alpha at each antenna's own IBO -- the
    per-antenna AGC term of mp_model.py:315-317 -- lies within the measurement's scatter
    (Rayleigh: 2.1e-4, the spread channel powers; LoS / two-path: 1.1e-5)."""
    import os
    import _engine
    a = np.loadtxt(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                "published_alpha_vs_tx_power_per_ant64_ibo0.0.csv"), delimiter=",")
    assert a.shape == (6, 64)
    for c, tol in ((0, 3e-4), (1, 2e-5), (2, 2e-5)):
        ibo, measured = a[2 * c], a[2 * c + 1]
        d = _engine.calc_alpha(ibo) - measured
        print("channel row", c, "max |diff|", np.abs(d).max(), "mean", d.mean())
        assert np.abs(d).max() <= tol


def test_calc_alpha_vs_reference_and_mpmath(units):
    """The float64 kernels' Bussgang gain outside the per-point fit (alpha_fit.h segment
    table, mimo_calc_alpha): the reference's own calc_alpha outputs (units.npz, NumPy /
    SciPy float64) within 4e-16 relative, and the 40-digit formula (mpmath) within 4e-16
    relative (2 ulp) from g = 0.002 to g = 7 (IBO -54 ... +17 dB; alpha = 1 from g 6.5 on)."""
    import _engine
    np.testing.assert_allclose(_engine.calc_alpha(units["alpha_ibo"]), units["alpha_out"], rtol=4e-16, atol=0)
    mpmath = pytest.importorskip("mpmath")
    mpmath.mp.dps = 40
    g = np.concatenate([np.geomspace(2e-3, 0.5, 300), np.linspace(0.5, 7.0, 1301)])
    ibo = 20.0 * np.log10(g)
    got = _engine.calc_alpha(ibo)
    worst = 0.0
    for g2, ai in zip(10.0 ** (ibo / 10.0), got):  # the float64 gamma^2 the host hands the kernel
        gm = mpmath.sqrt(mpmath.mpf(float(g2)))
        ref = 1 - mpmath.exp(-gm * gm) + mpmath.sqrt(mpmath.pi) / 2 * gm * mpmath.erfc(gm)
        worst = max(worst, float(abs((mpmath.mpf(float(ai)) - ref) / ref)))
    print("max relative error vs mpmath", worst)
    assert worst <= 4e-16


@pytest.mark.parametrize("F,S,cp", [(128, 64, 4), (2048, 1024, 128)])
def test_ofdm_tx_rx(units, F, S, cp):
    import modulation
    mod = modulation.OfdmQamModem(64, F, S, cp)
    td = mod.modulate(units[f"ofdm_bits_{F}"])
    np.testing.assert_allclose(td, units[f"ofdm_td_{F}"], rtol=1e-9, atol=1e-13)
    np.testing.assert_allclose(mod.demodulate(td, get_symbols_only=True), units[f"ofdm_rxsym_{F}"], rtol=1e-9,
                               atol=1e-12)
    np.testing.assert_array_equal(mod.demodulate(td), units[f"ofdm_rxbits_{F}"])


def test_array_transmit_and_receivers(units):
    link, mod = build_link(n_ant=4, n_sc=64, n_fft=128, M=16, ibo=2.0)
    link.my_miso_chan.channel_mat_fd = units["arr_H"]
    link.my_array.set_precoding_matrix(channel_mat_fd=units["arr_H"], mr_precoding=True)  # GPU MRT
    np.testing.assert_allclose(link.my_array.get_precoding_mat(), units["arr_P"], rtol=1e-12)
    link.recalculate_agc(channel_mat_fd=units["arr_H"])
    bits = units["arr_bits"]
    np.testing.assert_allclose(link.my_array.transmit(bits, out_domain_fd=True, skip_dist=False), units["arr_tx_fd"],
                               rtol=1e-9, atol=1e-13)
    np.testing.assert_allclose(link.my_array.transmit(bits, out_domain_fd=True, skip_dist=True),
                               units["arr_tx_fd_clean"], rtol=1e-9, atol=1e-13)
    res = link.my_cnc_rx.receive(n_iters_lst=units["cnc_iters"], in_sig_fd=units["cnc_in"])
    for i, b in enumerate(res):
        np.testing.assert_array_equal(b, units["cnc_bits"][i])
    mlink, _ = build_link(n_ant=4, n_sc=64, n_fft=128, M=16, ibo=2.0, is_mcnc=True)
    mlink.my_miso_chan.channel_mat_fd = units["arr_H"]
    mlink.my_cnc_rx.channel = mlink.my_miso_chan
    mlink.set_precoding_and_recalculate_agc()
    resm = mlink.my_cnc_rx.receive(n_iters_lst=units["mcnc_iters"], in_sig_fd=units["cnc_in"])
    for i, b in enumerate(resm):
        np.testing.assert_array_equal(b, units["mcnc_bits"][i])


def test_propagate_and_count():
    import channel
    import utilities
    rng = np.random.default_rng(0)
    h = rng.normal(size=(8, 128)) + 1j * rng.normal(size=(8, 128))
    y = rng.normal(size=(8, 128)) + 1j * rng.normal(size=(8, 128))
    ch = channel.MisoLosFd()
    ch.channel_mat_fd = h
    np.testing.assert_allclose(ch.propagate(y), np.sum(h * y, axis=0), rtol=1e-12)
    a = rng.integers(0, 2, 10000)
    b = rng.integers(0, 2, 10000)
    assert utilities.count_mismatched_bits(a, b) == int(np.bitwise_xor(a, b).sum())


def test_awgn_power():
    import noise
    n = noise.Awgn(snr_db=10.0, seed=3)
    x = np.zeros(200000, complex)
    y = n.process(x, avg_sample_pow=2.0)
    # E|n|^2 = P / snr  (noise.py:59-66)
    assert np.mean(np.abs(y) ** 2) == pytest.approx(0.2, rel=0.02)
    y2 = n.process(x, avg_sample_pow=2.0)
    assert not np.allclose(y, y2)


def test_cnc_receive_corrected_symbols(units):
    """CncReceiver.receive(return_bits=False) returns, per listed iteration, the corrected
    in-band symbols the slicer saw, rx - d (corrector.py:80-84), from the GPU CNC stage
    (mimo_cnc_receive_ex, ABI 7) -- against the oracle's restatement of the same loop."""
    import distortion
    from oracle import refmath as rm
    link, mod = build_link(n_ant=4, n_sc=64, n_fft=128, M=16, ibo=2.0)
    rx = link.my_cnc_rx
    iters = list(units["cnc_iters"])
    got = rx.receive(n_iters_lst=iters, in_sig_fd=units["cnc_in"], return_bits=False)
    kind, sat, p, toi = distortion.pa_params(rx.impairment)
    want = rm.cnc_receive(iters, np.asarray(units["cnc_in"])[rm.inband_bins(128, 64)], rm.gray_qam_constellation(16),
                          128, kind, sat, p, toi, rx.modem.alpha, return_bits=False)
    assert len(got) == len(sorted(set(iters)))
    for i, it in enumerate(sorted(set(int(v) for v in iters))):
        assert got[i].shape == (64,) and np.iscomplexobj(got[i])
        np.testing.assert_allclose(got[i], want[it], rtol=1e-9, atol=1e-10)
    # iteration 0 is the received in-band vector itself
    if 0 in iters:
        np.testing.assert_allclose(got[0], np.asarray(units["cnc_in"])[rm.inband_bins(128, 64)], rtol=0, atol=0)
    # and the bits path still agrees with the reference's fixture
    for i, b in enumerate(rx.receive(n_iters_lst=iters, in_sig_fd=units["cnc_in"])):
        np.testing.assert_array_equal(b, units["cnc_bits"][i])
