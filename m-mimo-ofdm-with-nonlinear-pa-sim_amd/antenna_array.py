"""Antenna arrays, precoding, PA calibration (reference antenna_array.py), MI355X build.

``transmit`` batches all antennas into one GPU call per stage (map, IFFT, PA, FFT)
instead of the reference's per-antenna Python loop (antenna_array.py:127-132), which
re-ran the QAM mapper once per antenna.  Single-user MRT precoding runs on the GPU.
Multi-user MR / ZF precoding (antenna_array.py:188-305) is not built:
set_precoding_matrix raises NotImplementedError for per-user channel lists.
"""
from __future__ import annotations

import copy
from abc import ABC
from typing import Union

import numpy as np
from numpy import ndarray

import _engine
import distortion
import utilities
from transceiver import Transceiver

SPEED_OF_LIGHT = 299792458.0


def sc_columns(channel_mat_fd, n_sc):
    """In-band columns [H[:, -S/2:], H[:, 1:S/2+1]] (antenna_array.py:163-164)."""
    h = np.asarray(channel_mat_fd)
    return np.concatenate((h[..., -(n_sc // 2):], h[..., 1:(n_sc // 2) + 1]), axis=-1)


class AntennaArray(ABC):
    """(antenna_array.py:13-412)"""

    def __init__(self, n_elements: int, base_transceiver: Transceiver, center_freq: int,
                 wav_len_spacing: float = 0.5, cord_x: float = 0, cord_y: float = 0, cord_z: float = 0):
        self.n_elements = n_elements
        self.n_users = base_transceiver.modem.n_users
        self.base_transceiver = base_transceiver
        self.center_freq = center_freq
        self.wav_len_spacing = wav_len_spacing
        self.array_elements = []
        self.cord_x = cord_x
        self.cord_y = cord_y
        self.cord_z = cord_z

    def set_tx_power_lvls(self, tx_power_dbm: float, total: bool = False) -> None:
        for tx in self.array_elements:
            tx.set_tx_power_dbm(10 * np.log10(10 ** (tx_power_dbm / 10) / len(self.array_elements)) if total
                                else tx_power_dbm)

    # ------------------------------------------------------------------ transmit
    def _uniform_pa(self):
        kinds = {distortion.pa_params(e.impairment) for e in self.array_elements}
        return next(iter(kinds)) if len(kinds) == 1 else None

    def transmit(self, in_bits: ndarray, out_domain_fd: bool = True, return_both: bool = False, skip_dist: bool = False,
                 sum_usr_signals: bool = True) -> Union[tuple, ndarray]:
        """Per-antenna precode -> OFDM -> PA (-> FFT): [A, F] or [A, F+cp] (antenna_array.py:58-140)."""
        sum_usr_signals = True  # one user (n_users > 1 is rejected by OfdmQamModem)
        modem = self.base_transceiver.modem
        pa = self._uniform_pa()
        if pa is None or not sum_usr_signals:
            return self._transmit_loop(in_bits, out_domain_fd, return_both, skip_dist, sum_usr_signals)
        sym = modem.modulate(in_bits, get_symbols_only=True)
        pre = np.stack([e.modem.precode_symbols(sym, e.modem.precoding_mat) for e in self.array_elements])
        clean_td = _engine.ofdm_tx(pre, modem.n_fft, modem.n_sub_carr, modem.cp_len)
        kind, sat, p, toi = pa
        dist_td = clean_td if (skip_dist or kind == "none") else _engine.pa(kind, clean_td, sat, p, toi)

        def fd(x):
            return _engine.fft(x[:, modem.cp_len:], inverse=False)

        out = fd(dist_td) if out_domain_fd else dist_td
        if return_both and not skip_dist:
            clean = fd(clean_td) if out_domain_fd else clean_td
            return np.squeeze(out), np.squeeze(clean)
        return np.squeeze(out)

    def _transmit_loop(self, in_bits, out_domain_fd, return_both, skip_dist, sum_usr_signals):
        res = [t.transmit(in_bits, out_domain_fd=out_domain_fd, return_both=return_both, skip_dist=skip_dist)
               for t in self.array_elements]
        if return_both and not skip_dist:
            return np.squeeze(np.stack([r[0] for r in res])), np.squeeze(np.stack([r[1] for r in res]))
        return np.squeeze(np.stack(res))

    # ------------------------------------------------------------------ precoding
    def set_precoding_matrix(self, channel_mat_fd=None, mr_precoding: bool = False, zf_precoding: bool = False,
                             update_distortion: bool = False, sep_carr_per_usr: bool = False) -> None:
        """(antenna_array.py:142-311)"""
        n_sc = self.base_transceiver.modem.n_sub_carr
        if isinstance(channel_mat_fd, list):
            # per-user channel lists: MU-MR / MU-ZF (antenna_array.py:188-305) are not part of
            # this build
            raise NotImplementedError("multi-user precoding is not supported by this build")
        hs = sc_columns(channel_mat_fd, n_sc)
        if mr_precoding:
            pm = _engine.mrt_precode(hs)
        else:
            pm = np.exp(1j * np.angle(np.conjugate(hs)))
        for idx, t in enumerate(self.array_elements):
            t.modem.set_precoding(pm[idx, :])
        if update_distortion:
            self.update_distortion(ibo_db=self.array_elements[0].impairment.ibo_db,
                                   avg_sample_pow=self.array_elements[0].modem.avg_sample_power)

    def _set_mrt_state(self, channel_mat_fd) -> None:
        """MRT precoding as object-state bookkeeping, host-side and HIP-free: ``Link``
        keeps the reference's attributes up to date with it at construction, before a
        driver forks (the per-trial MRT of the hot path runs on the device)."""
        hs = sc_columns(channel_mat_fd, self.base_transceiver.modem.n_sub_carr)
        pm = np.conjugate(hs) / np.sqrt(np.sum(np.abs(hs) ** 2, axis=0))
        for idx, t in enumerate(self.array_elements):
            t.modem.set_precoding(pm[idx, :])

    def update_distortion(self, ibo_db: float, avg_sample_pow: float, alpha_val: float = None) -> None:
        """Keep the IBO constant under precoding gain (antenna_array.py:313-360).

        gamma = mean |P|^2 over the whole [A, S] precoding matrix (an element without one
        counts as ones), summed per element (|P_a|^2 as one dot product each) instead of
        materialising the matrix, and the Bussgang gain formed once for the elements' common
        IBO: a 915-point grid calls this once per IBO on the timed host path (sweep.run_grid;
        2.7 -> 0.4 ms per call at 64 antennas)."""
        n_sc = self.base_transceiver.modem.n_sub_carr
        tot = 0.0
        for t in self.array_elements:
            p = t.modem.precoding_mat
            tot += float(n_sc) if p is None else float(np.vdot(p, p).real)
        gain = tot / (len(self.array_elements) * n_sc)
        alphas = {}  # per modem class (the elements are copies of one base transceiver)
        for t in self.array_elements:
            if isinstance(t.impairment, distortion.ThirdOrderNonLin):
                t.modem.alpha = alpha_val
                t.impairment.set_toi(ibo_db)
            else:
                k = type(t.modem)
                if k not in alphas:
                    alphas[k] = t.modem.calc_alpha(ibo_db=ibo_db)
                t.modem.alpha = alphas[k]
                t.impairment.set_ibo(ibo_db)
            t.impairment.set_avg_sample_power(avg_sample_pow * gain)

    def get_avg_precoding_gain(self) -> float:
        if self.n_users == 1:
            return float(np.average(np.abs(self.get_precoding_mat()) ** 2))
        return float(np.average(np.sum(np.abs(self.get_precoding_mat()) ** 2, axis=1)))

    def get_precoding_mat(self) -> ndarray:
        if self.n_users == 1:
            return np.stack([t.modem.precoding_mat for t in self.array_elements])
        return np.stack([t.modem.precoding_mat for t in self.array_elements])  # [tx, usr, sc]

    def update_n_users(self, n_users) -> None:
        self.n_users = n_users
        for t in self.array_elements:
            t.modem.n_users = n_users

    def positions(self) -> ndarray:
        return np.asarray([[t.cord_x, t.cord_y, t.cord_z] for t in self.array_elements], dtype=np.float64)


class LinearArray(AntennaArray):
    """ULA along x (antenna_array.py:415-445)."""

    def __init__(self, n_elements: int, base_transceiver: Transceiver, center_freq: int, wav_len_spacing: float,
                 cord_x: float = 0, cord_y: float = 0, cord_z: float = 0):
        super().__init__(n_elements, base_transceiver, center_freq, wav_len_spacing, cord_x, cord_y, cord_z)
        lam = SPEED_OF_LIGHT / self.center_freq
        half = (self.n_elements - 1) * self.wav_len_spacing * lam / 2
        for x in np.linspace(-half, half, self.n_elements):
            t = copy.deepcopy(self.base_transceiver)
            t.cord_x, t.cord_y, t.cord_z = x, 0, self.cord_z
            self.array_elements.append(t)


class CircularArray(AntennaArray):
    """UCA on a semicircle (antenna_array.py:448-479; the reference passes the wrong
    keyword names to pts_on_semicircum and cannot build one -- fixed here)."""

    def __init__(self, n_elements: int, base_transceiver: Transceiver, center_freq: int, wav_len_spacing: float,
                 cord_x: float = 0, cord_y: float = 0, cord_z: float = 0):
        super().__init__(n_elements, base_transceiver, center_freq, wav_len_spacing, cord_x, cord_y, cord_z)
        lam = SPEED_OF_LIGHT / self.center_freq
        radius = lam * (self.n_elements - 1) / (2 * np.pi)
        pts = utilities.pts_on_semicircum(radius=radius, n_points=self.n_elements)
        for idx in range(self.n_elements):
            t = copy.deepcopy(self.base_transceiver)
            t.cord_x, t.cord_y, t.cord_z = pts[idx][0], pts[idx][1], self.cord_z
            self.array_elements.append(t)


class PlanarRectangularArray(AntennaArray):
    """URA on the x-z plane (antenna_array.py:482-520)."""

    def __init__(self, n_elements_per_row: int, n_elements_per_col: int, base_transceiver: Transceiver,
                 center_freq: int, wav_len_spacing: float, cord_x: float = 0, cord_y: float = 0, cord_z: float = 0):
        super().__init__(n_elements_per_row * n_elements_per_col, base_transceiver, center_freq, wav_len_spacing,
                         cord_x, cord_y, cord_z)
        lam = SPEED_OF_LIGHT / self.center_freq
        col = np.linspace(-(n_elements_per_col - 1) * wav_len_spacing * lam / 2,
                          (n_elements_per_col - 1) * wav_len_spacing * lam / 2, n_elements_per_col)
        row = np.linspace(-(n_elements_per_row - 1) * wav_len_spacing * lam / 2,
                          (n_elements_per_row - 1) * wav_len_spacing * lam / 2, n_elements_per_row)
        for c in col:
            for r in row:
                t = copy.deepcopy(self.base_transceiver)
                t.cord_x, t.cord_y, t.cord_z = c, 0, self.cord_z + r
                self.array_elements.append(t)
