"""Pin the CPU oracle (oracle/) against the reference's own outputs (tests/golden/*.npz).

The fixtures were produced by ``tests/golden/make_golden.py`` running the reference
library in the build container (float64 / torch CPU FFT).  Integer paths must match
exactly; float paths to 1e-9 relative (torch pocketfft vs numpy pocketfft ordering).
"""
import numpy as np
import pytest

from conftest import link_fixture_names, load_golden, sim_config_from_fixture
from oracle import philox, refmath as rm, sim

RTOL = 1e-9


@pytest.mark.parametrize("M", [4, 16, 64, 256])
def test_constellation_and_modulate(units, M):
    c = rm.gray_qam_constellation(M)
    np.testing.assert_array_equal(c, units[f"const_{M}"])
    np.testing.assert_array_equal(rm.modulate(c, units[f"mod_bits_{M}"]), units[f"mod_out_{M}"])


@pytest.mark.parametrize("M", [4, 16, 64, 256])
def test_hard_demod_incl_ties(units, M):
    c = units[f"const_{M}"]
    z = units[f"demod_in_{M}"]
    np.testing.assert_array_equal(rm.demodulate(c, z), units[f"demod_bits_{M}"])
    np.testing.assert_array_equal(c[rm.detect_labels(c, z)], units[f"symdet_{M}"])


def test_llr(units):
    out = rm.soft_llr(units["const_16"], units["llr_in"], 0.7)
    np.testing.assert_allclose(out, units["llr_out"], rtol=1e-9, atol=1e-12)


def test_alpha(units):
    np.testing.assert_allclose(rm.calc_alpha(units["alpha_ibo"]), units["alpha_out"], rtol=1e-13)


def test_pa_models(units):
    x = units["pa_in"]
    np.testing.assert_allclose(rm.soft_limiter(float(units["pa_softlim_sat"]), x), units["pa_softlim_out"], rtol=1e-13)
    assert float(units["pa_softlim_sat"]) == pytest.approx(rm.sat_pow(3, 20.95), rel=1e-15)
    for p in (3, 4, 5):
        np.testing.assert_allclose(rm.rapp(rm.sat_pow(3, 20.95), p, x), units[f"pa_rapp{p}_out"], rtol=1e-13)
    coeff = rm.toi_coeff(12, 20.95)
    assert coeff == pytest.approx(float(units["pa_toi_coeff"]), rel=1e-15)
    np.testing.assert_allclose(rm.toi(coeff, x), units["pa_toi_out"], rtol=1e-13)


@pytest.mark.parametrize("F,S,cp", [(128, 64, 4), (2048, 1024, 128)])
def test_ofdm_tx_rx(units, F, S, cp):
    c = units["const_64"]
    sym = rm.modulate(c, units[f"ofdm_bits_{F}"])
    td = rm.ofdm_tx(sym, F, S, cp)
    np.testing.assert_allclose(td, units[f"ofdm_td_{F}"], rtol=RTOL, atol=1e-12)
    np.testing.assert_allclose(rm.ofdm_rx(td, F, S, cp), units[f"ofdm_rxsym_{F}"], rtol=RTOL, atol=1e-12)
    np.testing.assert_array_equal(rm.demodulate(c, rm.ofdm_rx(td, F, S, cp)), units[f"ofdm_rxbits_{F}"])


def test_precoding_agc_transmit(units):
    A, S, F, M = 4, 64, 128, 16
    c = units["const_16"]
    hs = rm.sc_channel(units["arr_H"], S)
    p = rm.mrt_precoding(hs)
    np.testing.assert_allclose(p, units["arr_P"], rtol=RTOL)
    avg = rm.ofdm_avg_sample_power(c, F, S)
    sat = rm.sat_pow(2.0, avg * rm.avg_precoding_gain(p))
    np.testing.assert_allclose(units["arr_sat"], sat, rtol=1e-13)
    g = rm.agc(hs, p, 2.0, S, A)
    bins = rm.inband_bins(F, S)
    np.testing.assert_allclose(units["arr_ak_agc"][bins], g["ak_hk_vk"], rtol=RTOL)
    np.testing.assert_allclose(units["arr_hk_agc"][bins], g["hk_vk"], rtol=RTOL)
    assert float(units["arr_ak_noise"]) == pytest.approx(g["ak_hk_vk_noise"], rel=1e-12)
    assert float(units["arr_hk_noise"]) == pytest.approx(g["hk_vk_noise"], rel=1e-12)
    s = rm.modulate(c, units["arr_bits"])
    fd = np.zeros((A, F), complex)
    fd[:, bins] = s[None, :] * p
    td = np.fft.ifft(fd, norm="ortho", axis=-1)
    np.testing.assert_allclose(np.fft.fft(rm.soft_limiter(sat, td), norm="ortho", axis=-1), units["arr_tx_fd"],
                               rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(np.fft.fft(td, norm="ortho", axis=-1), units["arr_tx_fd_clean"], rtol=1e-9, atol=1e-12)


def test_cnc_receiver(units):
    c = units["const_16"]
    S, F = 64, 128
    z = units["cnc_in"][rm.inband_bins(F, S)]
    out = rm.cnc_receive(units["cnc_iters"], z, c, F, "softlim", float(units["cnc_sat"]), 0, 0,
                         float(units["cnc_alpha"]))
    for i, it in enumerate(units["cnc_iters"]):
        np.testing.assert_array_equal(rm.labels_to_bits(out[int(it)], 4), units["cnc_bits"][i])


def test_mcnc_receiver(units):
    A, S, F, M = 4, 64, 128, 16
    c = units["const_16"]
    hs = rm.sc_channel(units["arr_H"], S)
    p = rm.mrt_precoding(hs)
    cfg = sim.SimConfig(A, S, F, M, pa="softlim", ibo_db=2.0, receiver="mcnc")
    pp = sim.point_params(cfg)
    g = rm.agc(hs, p, 2.0, S, A)
    z = units["cnc_in"][rm.inband_bins(F, S)]
    out = sim.mcnc_receive(cfg, [int(i) for i in units["mcnc_iters"]], z, c, p, hs, g["ak_hk_vk"], pp,
                           rm.avg_precoding_gain(p))
    for i, it in enumerate(units["mcnc_iters"]):
        np.testing.assert_array_equal(rm.labels_to_bits(out[int(it)], 4), units["mcnc_bits"][i])


def test_geometry_and_channels(units):
    pos = rm.ula_positions(4, 3.5e9, 0.5, 15)
    np.testing.assert_allclose(pos[:, 0], units["ula_x"], rtol=1e-15)
    rx = (212.0, 212.0, 1.5)
    np.testing.assert_allclose(rm.los_channel(pos, rx, 128, 15e3, 3.5e9), units["los_H"], rtol=1e-9)
    np.testing.assert_allclose(rm.two_path_channel(pos, rx, 128, 15e3, 3.5e9), units["twopath_H"], rtol=1e-9)
    np.testing.assert_allclose(rm.fspl_matrix(pos, rx, 128, 15e3, 3.5e9), units["rayleigh_att"], rtol=1e-12)
    np.testing.assert_allclose(rm.ebn0_to_snr(np.arange(0, 31.0), 1024, 1024, 64), units["ebn0_to_snr"], rtol=1e-14)


@pytest.mark.parametrize("name", link_fixture_names())
def test_link_end_to_end(name):
    """Oracle per-trial, per-iteration bit errors == reference Link.simulate on the same draws."""
    g = load_golden(f"link_{name}.npz")
    cfg = sim_config_from_fixture(g)
    seed, n = int(g["seed"]), int(g["n_trials"])
    d = sim.draws(cfg, seed, np.arange(n))
    assert int(d["labels"].sum()) == int(g["labels_sum"])  # the Philox streams are unchanged
    assert float(np.abs(d["z_chan"]).sum()) == pytest.approx(float(g["zchan_abs_sum"]), rel=1e-12)
    counts, dbg = [], None
    for j in range(n):
        c, dd = sim.run_trial(cfg, d["labels"][j], d["z_chan"][j], d["z_noise"][j], d["loc_u"][j],
                              d["z_csi"][j] if "z_csi" in d else None, g["iters"], bool(g["incl_clean"]),
                              return_debug=True)
        counts.append(c)
        if j == 0:
            dbg = dd
    np.testing.assert_allclose(dbg["z"], g["z_trial0"], rtol=1e-8, atol=1e-10)
    np.testing.assert_array_equal(np.asarray(counts), g["counts"])


@pytest.mark.parametrize("ebn0", [4.0, 8.0])
def test_config1_siso_awgn_on_cpu_path(ebn0):
    """BASELINE config 1 on the NumPy CPU path (no GPU): 1 antenna, 64 sub-carriers
    (FFT 128), 16-QAM, ideal PA (IBO 100 dB), LoS with the RX jitter -- an AWGN link after
    MRT / AGC.  The BASELINE run is 1e4 bits (40 symbols); 2e5 bits here for a tight check
    against Gray 16-QAM: BER = 3/8 erfc(sqrt(0.4 Eb/N0))."""
    from scipy import special
    from oracle import sim
    snr = float(sim.rm.ebn0_to_snr(ebn0, 64, 64, 16))
    cfg = sim.SimConfig(1, 64, 128, 16, pa="softlim", ibo_db=100.0, snr_db=snr, channel="los")
    counts = sim.run_trials(cfg, 11, np.arange(782), iters=[0], incl_clean=True)  # 782 x 256 bits ~ 2e5
    bits = 782 * 256
    ber = counts.sum(0) / bits
    theory = 3 / 8 * special.erfc(np.sqrt(0.4 * 10 ** (ebn0 / 10)))
    sigma = np.sqrt(theory * 4 / bits)
    assert np.all(np.abs(ber - theory) < 5 * sigma), (ber, theory)
    first40 = sim.run_trials(cfg, 11, np.arange(40), iters=[0])  # the BASELINE 1e4-bit run
    assert first40.shape == (40, 1) and 0 < first40.sum() < 40 * 256 * 0.2
