"""PA nonlinearity models (reference distortion.py), MI355X build: ``process`` runs on the GPU.

Same classes, attributes, setters and ``__str__`` as the reference, including
``Rapp.set_avg_sample_power`` not storing ``avg_samp_pow`` (distortion.py:165).
"""
from __future__ import annotations

import numpy as np
from numpy import ndarray

import _engine


class SoftLimiter:
    """Soft limiter / clipper (distortion.py:22-98)."""

    def __init__(self, ibo_db: float, avg_samp_pow: float):
        self.ibo_db = ibo_db
        self.avg_samp_pow = avg_samp_pow
        self.sat_pow = np.power(10, ibo_db / 10) * avg_samp_pow

    def __str__(self):
        return "softlim"

    def set_ibo(self, ibo_db: float) -> None:
        self.ibo_db = ibo_db
        self.sat_pow = np.power(10, ibo_db / 10) * self.avg_samp_pow

    def set_avg_sample_power(self, avg_samp_pow: float) -> None:
        self.avg_samp_pow = avg_samp_pow
        self.sat_pow = np.power(10, self.ibo_db / 10) * avg_samp_pow

    def process(self, in_sig: ndarray) -> ndarray:
        """y = x if |x|^2 <= sat else x sqrt(sat/|x|^2)  (distortion.py:9-19)."""
        return _engine.pa("softlim", in_sig, sat_pow=self.sat_pow)

    def plot_characteristics(self, *a, **k):
        raise NotImplementedError("plotting is out of scope of the MI355X engine")


class Rapp:
    """Rapp PA model (distortion.py:116-198)."""

    def __init__(self, ibo_db: float, avg_samp_pow: float, p_hardness: float):
        self.p_hardness = p_hardness
        self.ibo_db = ibo_db
        self.avg_samp_pow = avg_samp_pow
        self.sat_pow = np.power(10, ibo_db / 10) * avg_samp_pow

    def __str__(self):
        return "rapp"

    def set_hardness(self, p_hardness: float) -> None:
        self.p_hardness = p_hardness

    def set_ibo(self, ibo_db: float) -> None:
        self.ibo_db = ibo_db
        self.sat_pow = np.power(10, ibo_db / 10) * self.avg_samp_pow

    def set_avg_sample_power(self, avg_samp_pow: float) -> None:
        # the reference does not store avg_samp_pow here (distortion.py:165)
        self.sat_pow = np.power(10, self.ibo_db / 10) * avg_samp_pow

    def process(self, in_sig: ndarray) -> ndarray:
        """x / (1 + (|x|/sqrt(sat))^(2p))^(1/(2p))  (distortion.py:102-113)."""
        return _engine.pa("rapp", in_sig, sat_pow=self.sat_pow, p_hardness=self.p_hardness)

    def plot_characteristics(self, *a, **k):
        raise NotImplementedError("plotting is out of scope of the MI355X engine")


class ThirdOrderNonLin:
    """Memoryless cubic polynomial (distortion.py:215-282)."""

    def __init__(self, toi_db: float, avg_samp_pow: float):
        self.avg_samp_pow = avg_samp_pow
        self.toi_db = toi_db
        self.cubic_dist_coeff = 1 / (np.power(10, (toi_db / 10))) / avg_samp_pow

    def __str__(self):
        return "toi"

    def set_toi(self, toi_db: float) -> None:
        self.toi_db = toi_db
        self.cubic_dist_coeff = 1 / (np.power(10, (toi_db / 10))) / self.avg_samp_pow

    def set_avg_sample_power(self, avg_samp_pow: float) -> None:
        self.avg_samp_pow = avg_samp_pow
        self.cubic_dist_coeff = 1 / (np.power(10, (self.toi_db / 10))) / avg_samp_pow

    def process(self, in_sig):
        """x - c x |x|^2  (distortion.py:202-211)."""
        return _engine.pa("toi", in_sig, toi_coeff=self.cubic_dist_coeff)

    def plot_characteristics(self, *a, **k):
        raise NotImplementedError("plotting is out of scope of the MI355X engine")


def pa_params(impairment):
    """(kind, sat_pow, p_hardness, toi_coeff) of a PA object, for the engine."""
    if impairment is None:
        return "none", 0.0, 0.0, 0.0
    if isinstance(impairment, SoftLimiter):
        return "softlim", float(impairment.sat_pow), 0.0, 0.0
    if isinstance(impairment, Rapp):
        return "rapp", float(impairment.sat_pow), float(impairment.p_hardness), 0.0
    if isinstance(impairment, ThirdOrderNonLin):
        return "toi", 0.0, 0.0, float(impairment.cubic_dist_coeff)
    raise TypeError(f"unsupported impairment {type(impairment).__name__}")
