"""Numeric utilities of the reference (utilities.py), MI355X build.

Array compute (FFTs, bit-error counts) runs on the GPU through the C ABI; bit packing,
dB conversions, geometry helpers and CSV I/O are host-side format work.
Plotting helpers of the reference are out of scope.
"""
from __future__ import annotations

import csv

import numpy as np
from numpy import ndarray

import _engine


def dec2bitarray(in_number, bit_width: int) -> ndarray:
    """MSB-first bits of an int or int array (utilities.py:18-32)."""
    if isinstance(in_number, (np.integer, int)):
        return decimal2bitarray(int(in_number), bit_width).copy()
    nums = np.asarray(in_number, dtype=np.int64).reshape(-1)
    shifts = np.arange(bit_width - 1, -1, -1)
    return ((nums[:, None] >> shifts[None, :]) & 1).astype(np.int8).reshape(-1)


def decimal2bitarray(number: int, bit_width: int) -> ndarray:
    """(utilities.py:35-51)"""
    shifts = np.arange(bit_width - 1, -1, -1)
    return ((int(number) >> shifts) & 1).astype(np.int8)


def bitarray2dec(in_bitarray: ndarray) -> int:
    """(utilities.py:54-67)"""
    b = np.asarray(in_bitarray, dtype=np.int64).reshape(-1)
    return int((b * (1 << np.arange(b.size - 1, -1, -1))).sum()) if b.size else 0


def td_signal_power(signal: ndarray) -> float:
    """(utilities.py:70-79)"""
    return float(np.mean(np.abs(signal) ** 2))


def fd_signal_power(signal: ndarray) -> float:
    """(utilities.py:82-91)"""
    return float(np.sum(np.abs(signal) ** 2))


def count_mismatched_bits(tx_bits_arr: ndarray, rx_bits_arr: ndarray) -> int:
    """sum(tx XOR rx) on the GPU (utilities.py:94-104)."""
    return _engine.count_bit_errors(tx_bits_arr, rx_bits_arr)


def ebn0_to_snr(eb_per_n0, n_fft: int, n_sub_carr: int, constel_size: int):
    """(utilities.py:107-118)"""
    return 10 * np.log10(10 ** (np.asarray(eb_per_n0) / 10) * n_sub_carr * np.log2(constel_size) / n_fft)


def snr_to_ebn0(snr, n_fft: int, n_sub_carr: int, constel_size: int):
    """(utilities.py:121-133)"""
    return 10 * np.log10(10 ** (np.asarray(snr) / 10) * (n_fft / (n_sub_carr * np.log2(constel_size))))


def to_db(samples):
    """(utilities.py:136-143)"""
    return 10 * np.log10(samples)


def pts_on_circum(radius: float, n_points: int = 100) -> list:
    """(utilities.py:146-155)"""
    return [(np.cos(2 * np.pi / n_points * x) * radius, np.sin(2 * np.pi / n_points * x) * radius)
            for x in range(0, n_points + 1)]


def pts_on_semicircum(radius: float, n_points: int = 100) -> list:
    """(utilities.py:158-167)"""
    return [(np.cos(np.pi / n_points * x) * radius, np.sin(np.pi / n_points * x) * radius)
            for x in range(0, n_points + 1)]


def pts_on_semisphere(radius: float, n_points: int = 100, center_x: float = 0, center_y: float = 0,
                      center_z: float = 0):
    """(utilities.py:170-192)"""
    az = np.deg2rad(np.linspace(0, 180, int(np.sqrt(n_points)), endpoint=True))
    el = np.deg2rad(np.linspace(0, 180, int(np.sqrt(n_points)), endpoint=True))
    pts = []
    for a in az:
        for e in el:
            pts.append((-radius * np.sin(e) * np.cos(a) + center_x, -radius * np.sin(e) * np.sin(a) + center_y,
                        -radius * np.cos(e) + center_z))
    return pts


def to_freq_domain(in_sig_td: ndarray, remove_cp: bool = True, cp_len: int = None) -> ndarray:
    """Drop CP, ortho FFT along the last axis, on the GPU (utilities.py:311-329)."""
    x = np.asarray(in_sig_td)
    if remove_cp:
        x = x[..., cp_len:]
    return _engine.fft(x, inverse=False)


def to_time_domain(in_sig_mat_fd: ndarray) -> ndarray:
    """Ortho IFFT along the last axis, on the GPU (utilities.py:332-339)."""
    return _engine.fft(np.asarray(in_sig_mat_fd), inverse=True)


def save_to_csv(data_lst: list, filename: str, directory: str = "figs/csv_results") -> None:
    """One row per vector, ``csv.writer.writerows`` (utilities.py:342-352); the reference
    writes to ``figs/csv_results`` relative to the working directory."""
    import os
    os.makedirs(directory, exist_ok=True)
    with open(os.path.join(directory, "%s.csv" % filename), "w", newline="") as f:
        csv.writer(f).writerows([list(np.asarray(row, dtype=np.float64).reshape(-1)) for row in data_lst])


def read_from_csv(filename: str, directory: str = "../figs/csv_results") -> list:
    """List of float rows, ``QUOTE_NONNUMERIC`` (utilities.py:355-365; the reference reads
    from ``../figs/csv_results``)."""
    import os
    with open(os.path.join(directory, "%s.csv" % filename), "r", newline="") as f:
        return list(csv.reader(f, quoting=csv.QUOTE_NONNUMERIC))


def print_progress_bar(iteration: int, total: int, prefix: str = "", suffix: str = "", decimals: int = 1,
                       length: int = 100, fill: str = "#", print_end: str = "\r") -> None:
    """(utilities.py:369-392)"""
    percent = ("{0:." + str(decimals) + "f}").format(100 * (iteration / float(total)))
    filled = int(length * iteration // total)
    print(f"\r{prefix} |{fill * filled + '-' * (length - filled)}| {percent}% {suffix}", end=print_end)
    if iteration == total:
        print()
