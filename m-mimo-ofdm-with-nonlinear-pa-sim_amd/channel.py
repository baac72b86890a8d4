"""Frequency-domain MISO channels (reference channel.py), MI355X build.

Same classes and call signatures.  ``propagate`` (sum over antennas of H * Y) runs on the
GPU.  Channel matrices are closed-form geometry (LoS / two-path) or PCG64 draws
(Rayleigh, reference semantics) computed on the host when a caller asks for them; the
Link hot path does not use them -- it regenerates the per-trial channel on the device.
QuaDRiGa / random-paths channels need MATLAB or a NumPy-1 API and are out of scope.
"""
from __future__ import annotations

import numpy as np
from numpy import ndarray

import _engine

SPEED_OF_LIGHT = 299792458.0  # scipy.constants.c


def carrier_freqs(n_fft: int, carrier_spacing, center_freq) -> ndarray:
    """``torch.fft.fftfreq(n_fft, d=1/n_fft).numpy() * df + fc`` (channel.py:52-53).

    torch's fftfreq is float32 and the Python-int operands keep the result float32, so the
    reference's carrier grid is float32-quantised; mirrored exactly (float64 output).
    """
    k = np.fft.fftfreq(n_fft, d=1 / n_fft).astype(np.float32)
    return (k * np.float32(carrier_spacing) + np.float32(center_freq)).astype(np.float64)


def _distances(tx_transceivers, rx_transceiver):
    tx = np.asarray([[t.cord_x, t.cord_y, t.cord_z] for t in tx_transceivers], dtype=np.float64)
    rx = np.asarray([rx_transceiver.cord_x, rx_transceiver.cord_y, rx_transceiver.cord_z], dtype=np.float64)
    return tx, rx, np.sqrt(np.sum((tx - rx) ** 2, axis=1))


def _propagate(channel_mat_fd, in_sig_mat, sum_signals):
    if sum_signals:
        h = np.asarray(channel_mat_fd, np.complex128)
        y = np.broadcast_to(np.asarray(in_sig_mat, np.complex128), h.shape)
        return _engine.combine(h, y)
    return np.multiply(in_sig_mat, channel_mat_fd)


class MisoLosFd:
    """(channel.py:11-89)"""

    def __init__(self):
        self.channel_mat_fd = None

    def __str__(self):
        return "los"

    def get_channel_mat_fd(self) -> ndarray:
        return self.channel_mat_fd

    def calc_channel_mat(self, tx_transceivers, rx_transceiver, skip_attenuation: bool = False) -> None:
        f = carrier_freqs(rx_transceiver.modem.n_fft, rx_transceiver.carrier_spacing, rx_transceiver.center_freq)
        _, _, d = _distances(tx_transceivers, rx_transceiver)
        gains = np.asarray([t.tx_ant_gain_db for t in tx_transceivers], dtype=np.float64)
        ph = np.exp(2j * np.pi * np.outer(d, f) / SPEED_OF_LIGHT)
        if skip_attenuation:
            self.channel_mat_fd = ph
        else:
            att = np.sqrt(np.power(10, (gains[:, None] + rx_transceiver.rx_ant_gain_db) / 10)) * \
                (SPEED_OF_LIGHT / (4 * np.pi * np.outer(d, f)))
            self.channel_mat_fd = ph * att

    def propagate(self, in_sig_mat: ndarray, sum_signals: bool = True) -> ndarray:
        return _propagate(self.channel_mat_fd, in_sig_mat, sum_signals)


class MisoTwoPathFd:
    """(channel.py:92-184): LoS + ground reflection with coefficient -1."""

    def __init__(self):
        self.channel_mat_fd = None

    def __str__(self):
        return "two_path"

    def get_channel_mat_fd(self) -> ndarray:
        return self.channel_mat_fd

    def calc_channel_mat(self, tx_transceivers, rx_transceiver, skip_attenuation: bool = False) -> None:
        f = carrier_freqs(rx_transceiver.modem.n_fft, rx_transceiver.carrier_spacing, rx_transceiver.center_freq)
        tx, rx, d_los = _distances(tx_transceivers, rx_transceiver)
        gains = np.asarray([t.tx_ant_gain_db for t in tx_transceivers], dtype=np.float64)
        horiz = np.sqrt((tx[:, 0] - rx[0]) ** 2 + (tx[:, 1] - rx[1]) ** 2)
        elev = np.arctan((tx[:, 2] + rx[2]) / horiz)
        d_sec = tx[:, 2] / np.sin(elev) + rx[2] / np.sin(elev)
        los = np.exp(2j * np.pi * np.outer(d_los, f) / SPEED_OF_LIGHT)
        sec = -1.0 * np.exp(2j * np.pi * np.outer(d_sec, f) / SPEED_OF_LIGHT)
        if not skip_attenuation:
            g = np.sqrt(np.power(10, (gains[:, None] + rx_transceiver.rx_ant_gain_db) / 10))
            los = los * g * (SPEED_OF_LIGHT / (4 * np.pi * np.outer(d_los, f)))
            sec = sec * g * (SPEED_OF_LIGHT / (4 * np.pi * np.outer(d_sec, f)))
        self.channel_mat_fd = los + sec

    def propagate(self, in_sig_mat: ndarray, sum_signals: bool = True) -> ndarray:
        return _propagate(self.channel_mat_fd, in_sig_mat, sum_signals)


class MisoRayleighFd:
    """(channel.py:187-292): i.i.d. CN(0,1) x free-space attenuation."""

    def __init__(self, tx_transceivers, rx_transceiver, seed: int = None):
        self.n_inputs = len(tx_transceivers)
        self.fd_samp_size = tx_transceivers[0].modem.n_fft
        self.seed = 1234 if seed is None else seed
        self.rng_gen = np.random.default_rng(self.seed)
        f = carrier_freqs(rx_transceiver.modem.n_fft, rx_transceiver.carrier_spacing, rx_transceiver.center_freq)
        _, _, d = _distances(tx_transceivers, rx_transceiver)
        gains = np.asarray([t.tx_ant_gain_db for t in tx_transceivers], dtype=np.float64)
        self.los_fd_att_mat = np.sqrt(np.power(10, (gains[:, None] + rx_transceiver.rx_ant_gain_db) / 10)) * \
            (SPEED_OF_LIGHT / (4 * np.pi * np.outer(d, f)))
        self.fd_att_mat = None
        self.set_channel_mat_fd()

    def __str__(self):
        return "rayleigh"

    def set_channel_mat_fd(self, channel_mat_fd: ndarray = None, skip_attenuation: bool = False) -> None:
        if channel_mat_fd is None:
            self.reroll_channel_coeffs(skip_attenuation)
        else:
            self.channel_mat_fd = channel_mat_fd

    def get_channel_mat_fd(self) -> ndarray:
        return self.channel_mat_fd

    def reroll_channel_coeffs(self, skip_attenuation: bool = False) -> None:
        c = self.rng_gen.standard_normal(size=(self.n_inputs, self.fd_samp_size * 2)).view(
            dtype=np.complex128) / np.sqrt(2.0)
        self.channel_mat_fd = c if skip_attenuation else np.multiply(c, self.los_fd_att_mat)

    def propagate(self, in_sig_mat: ndarray, sum_signals: bool = True) -> ndarray:
        return _propagate(self.channel_mat_fd, in_sig_mat, sum_signals)
