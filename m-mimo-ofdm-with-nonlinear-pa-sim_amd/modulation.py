"""Modem / QAM / OFDM (reference modulation.py), MI355X build.

The QAM map, hard / soft demap and the OFDM IFFT/FFT run as float64 GPU stage kernels
(bit-exact labels vs the reference's argmin, including its lowest-label tie-break).
The device slicer handles the Gray square-QAM constellations ``QamModem`` builds, also
after ``correct_constellation`` scales them by alpha; any other constellation raises.
"""
from __future__ import annotations

import numpy as np
from numpy import ndarray
from scipy import special as scp_special

import _engine
from utilities import dec2bitarray, td_signal_power


def _gray_qam(constel_size: int) -> ndarray:
    L = int(round(np.sqrt(constel_size)))
    pam = np.arange(-L + 1, L, 2)
    lattice = np.tile(np.hstack((pam, pam[::-1])), L // 2) * 1j + pam.repeat(L)
    gray = np.asarray([x ^ (x >> 1) for x in range(constel_size)])
    return lattice[gray.argsort()]


def _qam_scale(constellation) -> float:
    """Real scale s with constellation == s * GrayQAM(M), else raise."""
    c = np.asarray(constellation)
    M = c.size
    L = int(round(np.sqrt(M)))
    if L * L != M or M & (M - 1) or M < 4:
        raise NotImplementedError("device QAM kernels handle square Gray QAM constellations only")
    ref = _gray_qam(M)
    s = float(np.real(c[-1] / ref[-1])) if ref[-1] != 0 else 1.0
    if not np.allclose(c, s * ref, rtol=1e-12, atol=1e-12):
        raise NotImplementedError("device QAM kernels handle (scaled) Gray square QAM constellations only")
    return s


def _labels(constellation, input_symbols) -> ndarray:
    s = _qam_scale(constellation)
    z = np.asarray(input_symbols, dtype=np.complex128).reshape(-1)
    return _engine.qam_slice(len(constellation), z / s if s != 1.0 else z)


def modulate(constellation: ndarray, n_bits_per_symbol: int, input_bits: ndarray) -> ndarray:
    """bits -> constellation[label] on the GPU (modulation.py:13-25)."""
    b = np.asarray(input_bits, dtype=np.int64).reshape(-1, n_bits_per_symbol)
    labels = (b * (1 << np.arange(n_bits_per_symbol - 1, -1, -1))).sum(axis=1)
    s = _qam_scale(constellation)
    out = _engine.qam_map(len(constellation), labels)
    return out * s if s != 1.0 else out


def soft_decoding(constellation: ndarray, n_bits_per_symbol: int, input_symbols: ndarray,
                  noise_var_vec: ndarray) -> ndarray:
    """LLR demodulation on the GPU (modulation.py:29-59)."""
    s = _qam_scale(constellation)
    z = np.asarray(input_symbols, np.complex128) / s
    return _engine.qam_llr(len(constellation), z, np.asarray(noise_var_vec, np.float64) / (s * s))


def demodulate(constellation: ndarray, n_bits_per_symbol: int, input_symbols: ndarray, soft: bool = False,
               noise_var: float = 0.0) -> ndarray:
    """Hard (argmin) or soft demodulation (modulation.py:63-88)."""
    if not soft:
        return dec2bitarray(_labels(constellation, input_symbols), n_bits_per_symbol)
    nv = noise_var if isinstance(noise_var, np.ndarray) else np.repeat(noise_var, len(input_symbols))
    return soft_decoding(constellation, n_bits_per_symbol, input_symbols, nv)


class Modem:
    """(modulation.py:91-220)"""

    def __init__(self, constellation: list, reorder_as_gray: bool = True):
        self.alpha = 1
        self.constel_size = len(constellation)
        if reorder_as_gray:
            gray_codes = np.asarray([x ^ (x >> 1) for x in range(self.constel_size)])
            self.constellation = np.array(constellation)[gray_codes.argsort()]
        else:
            self.constellation = constellation

    def modulate(self, input_bits: ndarray) -> ndarray:
        return modulate(self._constellation, self.n_bits_per_symbol, input_bits)

    def demodulate(self, input_symbols: ndarray) -> ndarray:
        return demodulate(self._constellation, self.n_bits_per_symbol, input_symbols)

    def symbol_detection(self, input_symbols: ndarray) -> ndarray:
        """(modulation.py:138-146)"""
        return self.constellation[_labels(self.constellation, input_symbols)]

    def correct_constellation(self, ibo_db: float) -> None:
        self.alpha = self.calc_alpha(ibo_db)
        self._constellation = self.alpha * self._constellation

    def calc_alpha(self, ibo_db):
        """Bussgang gain (modulation.py:178-189)."""
        gamma = np.power(10, ibo_db / 20)
        return 1 - np.exp(-np.power(gamma, 2)) + (np.sqrt(np.pi) * gamma / 2) * scp_special.erfc(gamma)

    def update_alpha(self, ibo_db: float) -> None:
        self.alpha = self.calc_alpha(ibo_db)

    def plot_constellation(self) -> None:
        raise NotImplementedError("plotting is out of scope of the MI355X engine")

    @property
    def constellation(self):
        return self._constellation

    @constellation.setter
    def constellation(self, constelation_symb_lst: list):
        n_bits_per_symbol = np.log2(len(constelation_symb_lst))
        if n_bits_per_symbol != int(n_bits_per_symbol):
            raise ValueError('Constellation length must be a power of 2.')
        self._constellation = np.array(constelation_symb_lst)
        self.avg_symbol_power = td_signal_power(self.constellation)
        self.constellation_size = self._constellation.size
        self.n_bits_per_symbol = int(n_bits_per_symbol)


class QamModem(Modem):
    """(modulation.py:223-244)"""

    def __init__(self, constel_size):
        n_symb = np.sqrt(constel_size)
        if n_symb != int(n_symb):
            raise ValueError('Constellation size must be a power of some number, only square QAM supported.')
        pam_symb = np.arange(-n_symb + 1, n_symb, 2)
        constellation = np.tile(np.hstack((pam_symb, pam_symb[::-1])), int(n_symb) // 2) * 1j + pam_symb.repeat(n_symb)
        super().__init__(constellation)


def _tx_ofdm_symbol(mod_symbols: ndarray, n_fft: int, n_sub_carr: int, cp_length: int) -> ndarray:
    """Bin map, ortho IFFT, CP on the GPU (modulation.py:248-273)."""
    if len(mod_symbols) != n_sub_carr:
        raise ValueError('mod_symbols length must match n_sub_carr value')
    return _engine.ofdm_tx(mod_symbols, n_fft, n_sub_carr, cp_length)


def _rx_ofdm_symbol(ofdm_symbol: ndarray, n_fft: int, n_sub_carr: int, cp_length: int) -> ndarray:
    """Drop CP, ortho FFT, in-band bins on the GPU (modulation.py:277-293)."""
    return _engine.ofdm_rx(ofdm_symbol, n_fft, n_sub_carr, cp_length)


class OfdmQamModem(QamModem):
    """(modulation.py:296-424)"""

    def __init__(self, constel_size: int, n_fft: int, n_sub_carr: int, cp_len: int, n_users: int = 1):
        super().__init__(constel_size)
        self.n_fft = n_fft
        self.n_sub_carr = n_sub_carr
        self.cp_len = cp_len
        self.n_bits_per_ofdm_sym = int(np.log2(constel_size) * n_sub_carr)
        self.avg_sample_power = self.ofdm_avg_sample_pow()
        self.precoding_mat = None
        if n_users != 1:
            # multi-user modulation / precoding (modulation.py:363-382, antenna_array.py:188-305)
            # is not part of this build: DESIGN.md §5 / §8
            raise NotImplementedError("multi-user OFDM (n_users > 1) is not supported by this build")
        self.n_users = n_users

    def set_precoding(self, precoding_mat: ndarray) -> None:
        self.precoding_mat = precoding_mat

    def precode_symbols(self, in_symbols: ndarray, precoding_mat: ndarray = None) -> ndarray:
        if precoding_mat is not None:
            return np.multiply(in_symbols, precoding_mat)
        return in_symbols

    def modulate(self, input_bits: ndarray, get_symbols_only: bool = False, sum_usr_signals: bool = True):
        """(modulation.py:346-382) one user: ``sum_usr_signals`` has nothing to sum."""
        sym = modulate(self._constellation, self.n_bits_per_symbol, input_bits)
        if get_symbols_only:
            return sym
        return _tx_ofdm_symbol(np.squeeze(self.precode_symbols(sym, self.precoding_mat)), self.n_fft,
                               self.n_sub_carr, self.cp_len)

    def demodulate(self, ofdm_symbol: ndarray, get_symbols_only: bool = False) -> ndarray:
        sym = _rx_ofdm_symbol(ofdm_symbol, self.n_fft, self.n_sub_carr, self.cp_len)
        if get_symbols_only:
            return sym
        return demodulate(self._constellation, self.n_bits_per_symbol, sym)

    def symbols_to_bits(self, input_symbols: ndarray) -> ndarray:
        return demodulate(self._constellation, self.n_bits_per_symbol, input_symbols)

    def soft_detection_llr(self, baseband_symbols, noise_var: float) -> ndarray:
        return demodulate(self._constellation, self.n_bits_per_symbol, baseband_symbols, soft=True,
                          noise_var=noise_var)

    def ofdm_avg_sample_pow(self) -> float:
        return self.avg_symbol_power * (self.n_sub_carr / self.n_fft)
