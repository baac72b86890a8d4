"""CPU (NumPy float64) restatement of the reference's hot-path arithmetic.

TEST INFRASTRUCTURE ONLY -- the oracle.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it; the product never does.

Every function states the reference file:line it follows (reference =
MarcinWachowiak/m-mimo-ofdm-with-nonlinear-pa-sim).  Parity of this restatement with
the reference itself is pinned by ``tests/test_oracle_golden.py`` against fixtures that
``tests/golden/make_golden.py`` captured by running the reference in the build
container.
"""
from __future__ import annotations

import numpy as np
from scipy import special as _sp


# --------------------------------------------------------------------------- QAM
def gray_qam_constellation(constel_size: int) -> np.ndarray:
    """Square QAM lattice re-ordered by Gray code.

    ``QamModem.__init__`` (modulation.py:230-244) builds the lattice
    ``tile(hstack(pam, pam[::-1])) * 1j + pam.repeat(L)``;
    ``Modem.__init__`` (modulation.py:110-114) reorders it with ``argsort`` of the Gray
    codes.  Closed form: C[label] = pam(g^-1(label >> h)) +
    j pam(g^-1(label & (2^h-1))).
    """
    L = int(round(np.sqrt(constel_size)))
    if L * L != constel_size:
        raise ValueError("Constellation size must be a power of some number, only square QAM supported.")
    if constel_size & (constel_size - 1):
        raise ValueError("Constellation length must be a power of 2.")
    pam = np.arange(-L + 1, L, 2).astype(np.float64)
    lattice = np.tile(np.hstack((pam, pam[::-1])), L // 2) * 1j + pam.repeat(L)
    gray = np.asarray([x ^ (x >> 1) for x in range(constel_size)])
    return lattice[gray.argsort()]


def bits_per_symbol(constel_size: int) -> int:
    return int(np.log2(constel_size))


def labels_to_bits(labels, n_bits: int) -> np.ndarray:
    """MSB-first expansion, ``utilities.dec2bitarray`` (utilities.py:18-51)."""
    labels = np.asarray(labels, dtype=np.int64).reshape(-1)
    shifts = np.arange(n_bits - 1, -1, -1)
    return ((labels[:, None] >> shifts[None, :]) & 1).astype(np.int8).reshape(-1)


def bits_to_labels(bits, n_bits: int) -> np.ndarray:
    """MSB-first packing, ``utilities.bitarray2dec`` (utilities.py:54-67) per symbol."""
    b = np.asarray(bits, dtype=np.int64).reshape(-1, n_bits)
    w = 1 << np.arange(n_bits - 1, -1, -1)
    return (b * w[None, :]).sum(axis=1)


def modulate(constellation, input_bits) -> np.ndarray:
    """``modulation.modulate`` (modulation.py:13-25): bits -> constellation[label]."""
    n_bits = bits_per_symbol(len(constellation))
    return np.asarray(constellation)[bits_to_labels(input_bits, n_bits)]


def detect_labels(constellation, symbols) -> np.ndarray:
    """Hard decision: ``argmin |z - C|`` with first-index tie-break.

    ``demodulate`` (modulation.py:75-76) and ``Modem.symbol_detection``
    (modulation.py:138-146).  Brute force on purpose: it is the oracle of the per-axis
    slicer the device uses.
    """
    symbols = np.asarray(symbols).reshape(-1)
    const = np.asarray(constellation)
    out = np.empty(symbols.shape[0], dtype=np.int64)
    step = 4096
    for i in range(0, symbols.shape[0], step):
        out[i:i + step] = np.abs(symbols[i:i + step] - const[:, None]).argmin(0)
    return out


def demodulate(constellation, symbols) -> np.ndarray:
    """``modulation.demodulate(soft=False)`` (modulation.py:75-77) -> bits."""
    return labels_to_bits(detect_labels(constellation, symbols), bits_per_symbol(len(constellation)))


def soft_llr(constellation, symbols, noise_var) -> np.ndarray:
    """``modulation.soft_decoding`` (modulation.py:29-59), vectorised.

    LLR of bit b (MSB-first position) = log(sum_{label bit=1} e^{-|z-C|^2/s2} /
    sum_{label bit=0} ...); +inf when the denominator underflows to 0.
    """
    const = np.asarray(constellation)
    n_bits = bits_per_symbol(len(const))
    symbols = np.asarray(symbols).reshape(-1)
    nv = np.broadcast_to(np.asarray(noise_var, dtype=np.float64), symbols.shape)
    metric = np.exp(-np.abs(symbols[:, None] - const[None, :]) ** 2 / nv[:, None])
    labels = np.arange(len(const))
    out = np.empty((symbols.shape[0], n_bits))
    for bit_index in range(n_bits):
        ones = ((labels >> bit_index) & 1).astype(bool)
        num = metric[:, ones].sum(axis=1)
        den = metric[:, ~ones].sum(axis=1)
        with np.errstate(divide="ignore"):
            val = np.where(den == 0, np.inf, np.log(np.abs(num) / np.where(den == 0, 1.0, np.abs(den))))
        out[:, n_bits - 1 - bit_index] = val
    return out.reshape(-1)


# --------------------------------------------------------------------------- OFDM
def inband_bins(n_fft: int, n_sub_carr: int) -> np.ndarray:
    """Sub-carrier k -> FFT bin (modulation.py:266-267, 293): negative half first, DC skipped."""
    half = n_sub_carr // 2
    return np.concatenate((np.arange(n_fft - half, n_fft), np.arange(1, half + 1)))


def ofdm_tx(symbols, n_fft: int, n_sub_carr: int, cp_len: int) -> np.ndarray:
    """``_tx_ofdm_symbol`` (modulation.py:248-273): map bins, ortho IFFT, prepend CP."""
    symbols = np.asarray(symbols)
    if symbols.shape[-1] != n_sub_carr:
        raise ValueError("mod_symbols length must match n_sub_carr value")
    fd = np.zeros(symbols.shape[:-1] + (n_fft,), dtype=np.complex128)
    fd[..., inband_bins(n_fft, n_sub_carr)] = symbols
    td = np.fft.ifft(fd, norm="ortho")
    return np.concatenate((td[..., n_fft - cp_len:], td), axis=-1)


def ofdm_rx(td, n_fft: int, n_sub_carr: int, cp_len: int) -> np.ndarray:
    """``_rx_ofdm_symbol`` (modulation.py:277-293): drop CP, ortho FFT, pick in-band bins."""
    fd = np.fft.fft(np.asarray(td)[..., cp_len:], norm="ortho")
    return fd[..., inband_bins(n_fft, n_sub_carr)]


def avg_symbol_power(constellation) -> float:
    """``td_signal_power(constellation)`` (modulation.py:218; utilities.py:70-79)."""
    return float(np.mean(np.abs(np.asarray(constellation)) ** 2))


def ofdm_avg_sample_power(constellation, n_fft, n_sub_carr) -> float:
    """``OfdmQamModem.ofdm_avg_sample_pow`` (modulation.py:418-424)."""
    return avg_symbol_power(constellation) * (n_sub_carr / n_fft)


def calc_alpha(ibo_db):
    """Bussgang gain of the soft limiter, ``Modem.calc_alpha`` (modulation.py:178-189)."""
    gamma = np.power(10.0, np.asarray(ibo_db, dtype=np.float64) / 20.0)
    return 1.0 - np.exp(-gamma ** 2) + (np.sqrt(np.pi) * gamma / 2.0) * _sp.erfc(gamma)


def ebn0_to_snr(eb_per_n0, n_fft, n_sub_carr, constel_size):
    """``utilities.ebn0_to_snr`` (utilities.py:107-118)."""
    return 10 * np.log10(10 ** (np.asarray(eb_per_n0) / 10) * n_sub_carr * np.log2(constel_size) / n_fft)


# --------------------------------------------------------------------------- PA models
def soft_limiter(sat_pow: float, x) -> np.ndarray:
    """``_process_soft_lim`` (distortion.py:9-19)."""
    x = np.asarray(x)
    p = np.abs(x) ** 2
    return np.where(p <= sat_pow, x, x * np.sqrt(sat_pow / np.abs(np.where(x != 0, x, 1)) ** 2))


def rapp(sat_pow: float, p_hardness: float, x) -> np.ndarray:
    """``_process_rapp`` (distortion.py:102-113)."""
    x = np.asarray(x)
    return x / np.power(1 + np.power(np.abs(x) / np.sqrt(sat_pow), 2 * p_hardness), 1 / (2 * p_hardness))


def toi(cubic_dist_coeff: float, x) -> np.ndarray:
    """``_process_toi`` (distortion.py:202-211)."""
    x = np.asarray(x)
    return x - cubic_dist_coeff * x * np.abs(x) ** 2


def sat_pow(ibo_db: float, avg_samp_pow: float) -> float:
    """``SoftLimiter``/``Rapp`` saturation power (distortion.py:37,51,61; 130,154,165)."""
    return float(np.power(10, ibo_db / 10) * avg_samp_pow)


def toi_coeff(toi_db: float, avg_samp_pow: float) -> float:
    """``ThirdOrderNonLin.cubic_dist_coeff`` (distortion.py:224,235,245)."""
    return float(1 / (np.power(10, (toi_db / 10))) / avg_samp_pow)


def apply_pa(kind: str, x, sat: float = 0.0, p_hardness: float = 0.0, coeff: float = 0.0):
    if kind == "softlim":
        return soft_limiter(sat, x)
    if kind == "rapp":
        return rapp(sat, p_hardness, x)
    if kind == "toi":
        return toi(coeff, x)
    if kind == "none":
        return np.asarray(x)
    raise ValueError(kind)


# --------------------------------------------------------------------------- precoding / AGC
def sc_channel(channel_mat_fd, n_sub_carr):
    """In-band columns ``[H[:, -S/2:], H[:, 1:S/2+1]]`` (antenna_array.py:163-164)."""
    h = np.asarray(channel_mat_fd)
    return np.concatenate((h[..., -(n_sub_carr // 2):], h[..., 1:(n_sub_carr // 2) + 1]), axis=-1)


def mrt_precoding(hs) -> np.ndarray:
    """Single-user MRT, ``set_precoding_matrix(mr_precoding=True)`` (antenna_array.py:165-173).

    ``P = conj(Hs) / sqrt(sum_ant |Hs|^2)`` for in-band ``Hs`` of shape [..., A, S].
    """
    hs = np.asarray(hs)
    return np.conjugate(hs) / np.sqrt(np.sum(np.abs(hs) ** 2, axis=-2, keepdims=True))


def phase_only_precoding(hs) -> np.ndarray:
    """``mr_precoding=False`` branch (antenna_array.py:175-178)."""
    return np.exp(1j * np.angle(np.conjugate(np.asarray(hs))))


def avg_precoding_gain(p) -> float:
    """``AntennaArray.update_distortion`` single-user gain (antenna_array.py:328-335)."""
    return float(np.average(np.abs(np.asarray(p)) ** 2))


def agc(hs, p, ibo_db, n_sub_carr, n_ant, alpha_fixed=None):
    """``Link.recalculate_agc`` (mp_model.py:290-329) for one trial.  ``alpha_fixed``: one
    gain for every antenna instead, as the TOI drivers' AGC (main_miso_cnc_ber_vs_ebn0_toi.py:247-259).

    Returns dict with ``hk_vk`` (clean-run gain, [S]), ``hk_vk_noise`` (scalar),
    ``alpha_vec`` ([A]), ``ak_hk_vk`` ([S]), ``ak_hk_vk_noise`` (scalar).
    """
    vk_pow = np.sum(np.abs(p) ** 2, axis=1)
    hk_vk = np.multiply(hs, p)
    hk_vk_avg = np.sum(hk_vk, axis=0)
    ibo_vec = 10 * np.log10(10 ** (ibo_db / 10) * n_sub_carr / (vk_pow * n_ant))
    ak = calc_alpha(ibo_vec)[:, None] if alpha_fixed is None else np.full((hs.shape[0], 1), float(alpha_fixed))
    ak_hk_vk_avg = np.sum(ak * hk_vk, axis=0)
    return dict(hk_vk=hk_vk_avg, hk_vk_noise=float(np.mean(np.abs(hk_vk_avg) ** 2)),
                alpha_vec=ak[:, 0], ak_hk_vk=ak_hk_vk_avg,
                ak_hk_vk_noise=float(np.mean(np.abs(ak_hk_vk_avg) ** 2)))


def csi_error(hs, eps, z_csi):
    """CSI-error model of ``Link.set_precoding_and_recalculate_agc`` (mp_model.py:264-282).

    ``Hhat = sqrt(1-eps^2) Hs + eps * sqrt(mean_k |Hs|^2) * z`` per antenna, z ~ CN(0,1).
    """
    pw = np.sum(np.abs(hs) ** 2, axis=-1, keepdims=True) / hs.shape[-1]
    return np.sqrt(1 - eps ** 2) * hs + z_csi * np.sqrt(pw) * eps


# --------------------------------------------------------------------------- channel geometry
SPEED_OF_LIGHT = 299792458.0


def fftfreq_carriers(n_fft, carrier_spacing, center_freq):
    """``torch.fft.fftfreq(n_fft, d=1/n_fft).numpy() * df + fc`` (channel.py:52-53).

    torch returns float32 and the Python-int operands keep it float32 (NumPy 2 weak
    scalars), so the reference's carrier frequencies are float32-quantised (256 Hz steps
    at 3.5 GHz).  Mirrored exactly: it moves LoS phases by up to ~1e-3 rad.
    """
    k = np.fft.fftfreq(n_fft, d=1 / n_fft).astype(np.float32)
    f = k * np.float32(carrier_spacing) + np.float32(center_freq)
    return f.astype(np.float64)


def fspl_matrix(tx_pos, rx_pos, n_fft, carrier_spacing, center_freq, gain_db=0.0):
    """Free-space attenuation ``sqrt(10^(G/10)) c / (4 pi d f)`` (channel.py:66-68, 223-225)."""
    tx_pos = np.asarray(tx_pos, dtype=np.float64)
    d = np.sqrt(np.sum((tx_pos - np.asarray(rx_pos, dtype=np.float64)) ** 2, axis=1))
    f = fftfreq_carriers(n_fft, carrier_spacing, center_freq)
    return np.sqrt(np.power(10, gain_db / 10)) * (SPEED_OF_LIGHT / (4 * np.pi * np.outer(d, f)))


def los_channel(tx_pos, rx_pos, n_fft, carrier_spacing, center_freq, gain_db=0.0):
    """``MisoLosFd.calc_channel_mat`` (channel.py:35-72)."""
    tx_pos = np.asarray(tx_pos, dtype=np.float64)
    d = np.sqrt(np.sum((tx_pos - np.asarray(rx_pos, dtype=np.float64)) ** 2, axis=1))
    f = fftfreq_carriers(n_fft, carrier_spacing, center_freq)
    ph = np.exp(2j * np.pi * np.outer(d, f) / SPEED_OF_LIGHT)
    att = np.sqrt(np.power(10, gain_db / 10)) * (SPEED_OF_LIGHT / (4 * np.pi * np.outer(d, f)))
    return ph * att


def two_path_channel(tx_pos, rx_pos, n_fft, carrier_spacing, center_freq, gain_db=0.0):
    """``MisoTwoPathFd.calc_channel_mat`` (channel.py:116-167): LoS + (-1) ground reflection."""
    tx_pos = np.asarray(tx_pos, dtype=np.float64)
    rx_pos = np.asarray(rx_pos, dtype=np.float64)
    f = fftfreq_carriers(n_fft, carrier_spacing, center_freq)
    d_los = np.sqrt(np.sum((tx_pos - rx_pos) ** 2, axis=1))
    horiz = np.sqrt((tx_pos[:, 0] - rx_pos[0]) ** 2 + (tx_pos[:, 1] - rx_pos[1]) ** 2)
    elev = np.arctan((tx_pos[:, 2] + rx_pos[2]) / horiz)
    d_sec = tx_pos[:, 2] / np.sin(elev) + rx_pos[2] / np.sin(elev)
    g = np.sqrt(np.power(10, gain_db / 10))
    los = np.exp(2j * np.pi * np.outer(d_los, f) / SPEED_OF_LIGHT) * g * SPEED_OF_LIGHT / (4 * np.pi * np.outer(d_los, f))
    sec = -1.0 * np.exp(2j * np.pi * np.outer(d_sec, f) / SPEED_OF_LIGHT) * g * SPEED_OF_LIGHT / (4 * np.pi * np.outer(d_sec, f))
    return los + sec


def ula_positions(n_elements, center_freq, wav_len_spacing=0.5, cord_z=0.0):
    """``LinearArray`` element placement (antenna_array.py:428-445).

    x = linspace(-(n-1) s lambda / 2, +(n-1) s lambda / 2), y = 0, z = cord_z (the
    reference ignores the array's cord_x / cord_y here).
    """
    wav_len = 299792458.0 / center_freq
    half = (n_elements - 1) * wav_len_spacing * wav_len / 2
    xs = np.linspace(-half, half, n_elements)
    return np.stack([xs, np.zeros(n_elements), np.full(n_elements, float(cord_z))], axis=1)


# --------------------------------------------------------------------------- receivers
def cnc_receive(n_iters_lst, rx_nsc, constellation, n_fft, pa_kind, sat, p_hardness, coeff, alpha,
                return_bits=True):
    """``CncReceiver.receive`` (corrector.py:52-112) on the in-band vector ``rx_nsc`` [S].

    Returns {iteration: detected labels}, or with ``return_bits=False`` {iteration: the
    corrected input ``rx - d`` the slicer saw} (corrector.py:80-84).
    """
    n_sc = rx_nsc.shape[-1]
    bins = inband_bins(n_fft, n_sc)
    const = np.asarray(constellation)
    out = {}
    d = None
    for it in range(int(np.max(n_iters_lst)) + 1):
        v = rx_nsc if it == 0 else rx_nsc - d
        lab = detect_labels(const, v)
        s_hat = const[lab]
        if it in set(int(i) for i in n_iters_lst):
            out[it] = lab if return_bits else v
        up = np.zeros(n_fft, dtype=np.complex128)
        up[bins] = s_hat
        td = np.fft.ifft(up, norm="ortho")
        td = apply_pa(pa_kind, td, sat, p_hardness, coeff)
        est = np.fft.fft(td, norm="ortho")[bins] / alpha
        d = est - s_hat
    return out
