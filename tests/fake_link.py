"""Deterministic stand-in for mp_model.Link on machines without a GPU: counters depend only
on (IBO, SNR, seed, counter index), so a sharded sweep must reproduce the single-process
grid exactly.  Used by the CPU gloo tests of sweep.run_grid and of bench.py's grid line."""
import numpy as np


class FakeModem:
    n_sub_carr, constel_size = 64, 16


class FakeLink:
    my_mod = FakeModem()

    def __init__(self):
        self.ibo = None
        self.snr = None

    def update_distortion(self, ibo_val_db):
        self.ibo = ibo_val_db

    def set_snr(self, snr_db_val):
        self.snr = snr_db_val

    def simulate(self, incl_clean, reroll, iters, seed_arr, err, bits):
        n = len(iters) + (1 if incl_clean else 0)
        for i in range(n):
            bits[i] += 256 * 100
            err[i] += int(1000 * np.exp(-0.2 * self.snr) * (1 + i) * (1 + self.ibo)) + seed_arr[1] % 3
