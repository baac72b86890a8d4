"""Per-antenna modem + PA (reference transceiver.py), MI355X build."""
from __future__ import annotations

import numpy as np
from numpy import ndarray

import distortion
import utilities
from modulation import OfdmQamModem


class Transceiver:
    """(transceiver.py:8-184)"""

    def __init__(self, modem: OfdmQamModem, center_freq: int, carrier_spacing: int, impairment, cord_x: float = 0,
                 cord_y: float = 0, cord_z: float = 0):
        self.modem = modem
        self.impairment = impairment
        self.center_freq = center_freq
        self.carrier_spacing = carrier_spacing
        if isinstance(impairment, distortion.SoftLimiter):
            self.modem.update_alpha(ibo_db=impairment.ibo_db)
        self.tx_ant_gain_db = 0
        self.rx_ant_gain_db = 0
        self.tx_power_dbm = 10 * np.log10(1000 * self.modem.avg_sample_power)
        self.cord_x = cord_x
        self.cord_y = cord_y
        self.cord_z = cord_z

    def set_position(self, cord_x: float, cord_y: float, cord_z: float) -> None:
        self.cord_x, self.cord_y, self.cord_z = cord_x, cord_y, cord_z

    def set_ant_gains(self, tx_ant_gain_db: float, rx_ant_gain_db: float) -> None:
        self.tx_ant_gain_db = tx_ant_gain_db
        self.rx_ant_gain_db = rx_ant_gain_db

    def set_tx_power_dbm(self, tx_power_dbm: float) -> None:
        self.tx_power_dbm = tx_power_dbm

    def correct_constellation(self) -> None:
        self.modem.correct_constellation(ibo_db=self.impairment.ibo_db)

    def update_distortion(self, ibo_db: float) -> None:
        self.impairment.set_ibo(ibo_db=ibo_db)
        self.modem.update_alpha(ibo_db=ibo_db)

    def transmit(self, in_bits: ndarray, out_domain_fd: bool = True, skip_dist: bool = False, return_both: bool = False,
                 sum_usr_signals: bool = True):
        """modulate -> PA -> (FFT)  (transceiver.py:98-174)."""
        clean = self.modem.modulate(in_bits, sum_usr_signals=sum_usr_signals)  # one user: nothing to sum
        sigs = [clean]

        def fd(x):
            return utilities.to_freq_domain(x, remove_cp=True, cp_len=self.modem.cp_len)

        out = []
        for c in sigs:
            if skip_dist or self.impairment is None:
                out.append(fd(c) if out_domain_fd else c)
            else:
                d = self.impairment.process(c)
                if return_both:
                    out.append([fd(d), fd(c)] if out_domain_fd else [d, c])
                else:
                    out.append(fd(d) if out_domain_fd else d)
        return tuple(out[0]) if (return_both and not skip_dist and self.impairment is not None) else out[0]

    def receive(self, in_symb_td: ndarray) -> ndarray:
        """OFDM demod + hard demap (transceiver.py:176-184)."""
        return self.modem.demodulate(in_symb_td)
