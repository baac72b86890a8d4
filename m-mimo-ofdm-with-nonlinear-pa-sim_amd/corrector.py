"""Clipping-noise-cancellation receivers (reference corrector.py), MI355X build.

``CncReceiver.receive`` runs the whole iteration loop as float64 GPU stage kernels;
``McncReceiver.receive`` composes the GPU array transmit and channel combine.  Inside
``Link.simulate`` both receivers run fused in the per-trial kernel instead.
Multi-user variants (corrector.py:248-489) are out of scope for this round.
"""
from __future__ import annotations

import numpy as np
from numpy import ndarray

import _engine
import distortion
from antenna_array import AntennaArray, sc_columns
from modulation import OfdmQamModem, _qam_scale


class CncReceiver:
    """(corrector.py:12-112)"""

    def __init__(self, modem: OfdmQamModem, impairment):
        self.modem = modem
        self.impairment = impairment
        if isinstance(self.impairment, distortion.SoftLimiter):
            self.modem.alpha = self.modem.calc_alpha(self.impairment.ibo_db)
        else:
            self.modem.alpha = 1.0
        self.upsample_factor = self.modem.n_fft / self.modem.n_sub_carr
        self.impairment.set_avg_sample_power(avg_samp_pow=self.modem.avg_symbol_power * (1 / self.upsample_factor))

    def update_distortion(self, ibo_db: float, alpha_val: float = 1.0) -> None:
        if isinstance(self.impairment, distortion.ThirdOrderNonLin):
            self.impairment.set_toi(ibo_db)
            self.modem.alpha = alpha_val
        else:
            self.impairment.set_ibo(ibo_db)
            self.modem.alpha = self.modem.calc_alpha(ibo_db)

    def receive(self, n_iters_lst: list, in_sig_fd: ndarray, alpha_estimate: float = None,
                return_bits: bool = True) -> list:
        n_sc = self.modem.n_sub_carr
        rx = sc_columns(in_sig_fd, n_sc)
        alpha = self.modem.alpha if alpha_estimate is None else alpha_estimate
        kind, sat, p, toi = distortion.pa_params(self.impairment)
        iters = sorted(set(int(i) for i in np.atleast_1d(n_iters_lst)))
        s = _qam_scale(self.modem.constellation)
        out = _engine.cnc_receive(self.modem.constel_size, self.modem.n_fft, kind, sat, p, toi, alpha, iters,
                                  rx / s if s != 1.0 else rx, return_bits=return_bits)
        if not return_bits:
            # the corrected in-band symbols the slicer saw (corrector.py:80-84), in the caller's scale
            return [out[i] * s if s != 1.0 else out[i] for i in iters]
        from utilities import dec2bitarray
        return [dec2bitarray(out[i], self.modem.n_bits_per_symbol) for i in iters]


class McncReceiver:
    """(corrector.py:115-245)"""

    def __init__(self, antenna_array: AntennaArray, channel, alpha_estimate: float = None, _host_setup=False):
        self.antenna_array = antenna_array
        self.channel = channel
        if _host_setup:  # Link construction: stay HIP-free before the drivers fork
            self.antenna_array._set_mrt_state(self.channel.get_channel_mat_fd())
        else:
            self.antenna_array.set_precoding_matrix(channel_mat_fd=self.channel.get_channel_mat_fd(), mr_precoding=True)
        self.n_sub_carr = self.antenna_array.array_elements[0].modem.n_sub_carr
        self.update_agc(alpha_estimate)

    def receive(self, n_iters_lst: list, in_sig_fd: ndarray, return_bits: bool = True) -> list:
        modem = self.antenna_array.array_elements[0].modem
        rx = sc_columns(in_sig_fd, self.n_sub_carr)
        iters = set(int(i) for i in np.atleast_1d(n_iters_lst))
        out = []
        d = None
        for it in range(int(np.max(n_iters_lst)) + 1):
            v = rx if it == 0 else rx - d
            s_hat = modem.symbol_detection(v)
            bits = modem.symbols_to_bits(s_hat)
            if it in iters:
                out.append(bits if return_bits else v)
            tx = self.antenna_array.transmit(bits, out_domain_fd=True, return_both=False)
            r = self.channel.propagate(in_sig_mat=tx) / self.agc_corr_vec
            d = sc_columns(r, self.n_sub_carr) - s_hat
        return out

    def update_agc(self, alpha_estimate: float = None) -> None:
        """(corrector.py:209-245)"""
        arr = self.antenna_array
        n_sc = self.n_sub_carr
        hk = sc_columns(self.channel.get_channel_mat_fd(), n_sc)
        vk = arr.get_precoding_mat()
        vk_pow = np.sum(np.abs(vk) ** 2, axis=1)
        hk_vk = hk * vk
        modem = arr.array_elements[0].modem
        if alpha_estimate is None and not isinstance(arr.array_elements[0].impairment, distortion.ThirdOrderNonLin):
            ibo_vec = 10 * np.log10(10 ** (arr.array_elements[0].impairment.ibo_db / 10) * n_sc /
                                    (vk_pow * len(arr.array_elements)))
            ak = modem.calc_alpha(ibo_db=ibo_vec)
        else:
            ak = np.repeat(alpha_estimate, len(arr.array_elements))
        g = np.sum(np.expand_dims(ak, 1) * hk_vk, axis=0)
        agc = np.ones(modem.n_fft, dtype=np.complex128)
        agc[-(n_sc // 2):] = g[:n_sc // 2]
        agc[1:(n_sc // 2) + 1] = g[n_sc // 2:]
        self.agc_corr_vec = agc
