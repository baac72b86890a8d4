"""AWGN (reference noise.py), MI355X build.

``Awgn.process`` draws its normals on the GPU from a Philox stream keyed by the object's
seed and a per-call counter (the reference draws PCG64 normals from ``rng_gen``,
noise.py:66); the scaling is the reference's: n = (x + jy) sqrt(2 P / snr) / 2.
"""
from __future__ import annotations

from abc import ABC

import numpy as np
from numpy import ndarray

import _engine
from utilities import fd_signal_power, to_db


class Noise(ABC):
    """(noise.py:8-27)"""

    def __init__(self, snr_db: float, noise_p_dbm: float, seed: int):
        self.snr_db = snr_db
        self.noise_p_dbm = noise_p_dbm
        self.seed = 1234 if seed is None else seed
        self.rng_gen = np.random.default_rng(self.seed)
        self._calls = 0


class Awgn(Noise):
    """(noise.py:30-83)"""

    def __init__(self, snr_db=None, noise_p_dbm=None, seed=None):
        super().__init__(snr_db, noise_p_dbm, seed)

    def process(self, in_sig: ndarray, avg_sample_pow: float = 1, fixed_noise_power: bool = False,
                disp_data: bool = False) -> ndarray:
        if fixed_noise_power:
            noise_std = np.sqrt(2 * 0.001 * 10 ** (self.noise_p_dbm / 10))
        else:
            noise_std = np.sqrt(2 * avg_sample_pow / (10 ** (self.snr_db / 10)))
        # the seed of this call's Philox stream follows the object's numpy generator, so
        # reseeding rng_gen (as Link.simulate does, mp_model.py:122) reseeds the noise
        key = int(self.rng_gen.integers(0, 2 ** 63))
        out = _engine.awgn(in_sig, float(noise_std), key, self._calls)
        self._calls += 1
        if disp_data:
            noise = out - np.asarray(in_sig)
            print("Signal power:[dBm]", to_db(fd_signal_power(in_sig) + 30))
            print("Noise power:[dBm]", to_db(fd_signal_power(noise)) + 30)
            print("SNR: ", to_db(fd_signal_power(in_sig) / fd_signal_power(noise)))
        return out
