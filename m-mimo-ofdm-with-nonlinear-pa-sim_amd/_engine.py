"""ctypes binding of libmimo_engine.so (include/mimo_engine.h).

This is the reference-side FFI a maintainer would add: plain pointers and sizes, no
torch types.  The library is built in-tree by ``__graft_entry__.build()`` (``make`` in
``csrc/``); there is no CPU fallback -- if the library or a GPU is missing, calls raise.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MIMO_LIB") or os.path.join(_HERE, "libmimo_engine.so")

PA_KINDS = {"none": 0, "softlim": 1, "rapp": 2, "toi": 3}
CH_KINDS = {"rayleigh": 1, "los": 2, "two_path": 3, "table": 4}
RX_KINDS = {"cnc": 1, "mcnc": 2}
# Arithmetic type of the fused kernel: "f64" is the reference's own precision (complex128 /
# float64, the default); "f32" is the fast variant.  MIMO_PRECISION overrides the default.
PRECISIONS = {"f64": 0, "f32": 1}


def default_precision():
    p = os.environ.get("MIMO_PRECISION", "f64").lower()
    if p not in PRECISIONS:
        raise ValueError(f"MIMO_PRECISION must be one of {sorted(PRECISIONS)}")
    return p

_dp = ctypes.POINTER(ctypes.c_double)
_i32p = ctypes.POINTER(ctypes.c_int32)
_i64p = ctypes.POINTER(ctypes.c_int64)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_u32p = ctypes.POINTER(ctypes.c_uint32)


class MimoConfig(ctypes.Structure):
    _fields_ = [("n_ant", ctypes.c_int32), ("n_sub_carr", ctypes.c_int32), ("n_fft", ctypes.c_int32),
                ("constel_size", ctypes.c_int32), ("cp_len", ctypes.c_int32), ("channel_kind", ctypes.c_int32),
                ("receiver_kind", ctypes.c_int32), ("device", ctypes.c_int32), ("rx_pos", ctypes.c_double * 3),
                ("rx_loc_var", ctypes.c_double), ("reroll_chan", ctypes.c_int32), ("precision", ctypes.c_int32),
                ("tx_pos", _dp), ("carrier_freqs", _dp), ("chan_table", _dp), ("chan_replay_period", ctypes.c_int32),
                ("csi_seed", ctypes.c_uint64)]


class MimoPoint(ctypes.Structure):
    _fields_ = [("ibo_db", ctypes.c_double), ("snr_db", ctypes.c_double), ("avg_symbol_power", ctypes.c_double),
                ("pa_kind", ctypes.c_int32), ("cnc_pa_kind", ctypes.c_int32), ("sat_pow", ctypes.c_double),
                ("p_hardness", ctypes.c_double), ("toi_coeff", ctypes.c_double), ("cnc_sat_pow", ctypes.c_double),
                ("cnc_toi_coeff", ctypes.c_double), ("cnc_alpha", ctypes.c_double), ("csi_eps", ctypes.c_double),
                ("array_alpha", ctypes.c_double)]


SYMBOLS = {
    "mimo_abi_version": (ctypes.c_int32, []),
    "mimo_last_error": (ctypes.c_char_p, []),
    "mimo_device_count": (ctypes.c_int32, []),
    "mimo_engine_create": (ctypes.c_void_p, [ctypes.POINTER(MimoConfig)]),
    "mimo_engine_set_point": (ctypes.c_int32, [ctypes.c_void_p, ctypes.POINTER(MimoPoint)]),
    "mimo_engine_run": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, _i32p,
                                         ctypes.c_int32, ctypes.c_int32, _u64p, _u64p, _u32p]),
    "mimo_engine_run_points": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(MimoPoint), _u64p,
                                                _u64p, _u64p, _i32p, ctypes.c_int32, ctypes.c_int32, _u64p, _u64p,
                                                _u32p]),
    "mimo_engine_last_kernel_ms": (ctypes.c_double, [ctypes.c_void_p]),
    "mimo_engine_describe": (ctypes.c_char_p, [ctypes.c_void_p]),
    "mimo_engine_destroy": (None, [ctypes.c_void_p]),
    "mimo_qam_map": (ctypes.c_int32, [ctypes.c_int32, _i32p, ctypes.c_int64, _dp]),
    "mimo_qam_slice": (ctypes.c_int32, [ctypes.c_int32, _dp, ctypes.c_int64, _i32p]),
    "mimo_qam_llr": (ctypes.c_int32, [ctypes.c_int32, _dp, ctypes.c_int64, _dp, _dp]),
    "mimo_fft": (ctypes.c_int32, [ctypes.c_int32, ctypes.c_int64, ctypes.c_int32, _dp, _dp]),
    "mimo_ofdm_tx": (ctypes.c_int32, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, _dp, _dp]),
    "mimo_ofdm_rx": (ctypes.c_int32, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, _dp, _dp]),
    "mimo_pa": (ctypes.c_int32, [ctypes.c_int32, ctypes.c_double, ctypes.c_double, ctypes.c_double, _dp,
                                 ctypes.c_int64, _dp]),
    "mimo_calc_alpha": (ctypes.c_int32, [_dp, ctypes.c_int64, _dp]),
    "mimo_mrt_precode": (ctypes.c_int32, [ctypes.c_int32, ctypes.c_int32, _dp, _dp]),
    "mimo_combine": (ctypes.c_int32, [ctypes.c_int32, ctypes.c_int64, _dp, _dp, _dp]),
    "mimo_awgn": (ctypes.c_int32, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int64, ctypes.c_double, _dp, _dp]),
    "mimo_count_bit_errors": (ctypes.c_int32, [_i64p, _i64p, ctypes.c_int64, _i64p]),
    "mimo_cnc_receive": (ctypes.c_int32, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                          ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double, _i32p,
                                          ctypes.c_int32, _dp, _i32p]),
    "mimo_cnc_receive_ex": (ctypes.c_int32, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                             ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double, _i32p,
                                             ctypes.c_int32, _dp, _i32p, _dp]),
}

_lib = None


class EngineError(RuntimeError):
    pass


ABI_VERSION = 8  # include/mimo_engine.h MIMO_ABI_VERSION


def lib():
    """Load the HIP engine library; raises if it was not built (no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise EngineError(f"{LIB_PATH} not found: build it with __graft_entry__.build() (make -C csrc)")
        handle = ctypes.CDLL(LIB_PATH)
        # the ABI first: the structures below are ABI 8's (mimo_point.array_alpha),
        # and a stale library lacks the newer entry points -- binding them first would raise a
        # bare AttributeError instead of this message
        ver = getattr(handle, "mimo_abi_version", None)
        if ver is None:
            raise EngineError(f"{LIB_PATH} exports no mimo_abi_version (older than ABI 2): rebuild it")
        ver.restype, ver.argtypes = ctypes.c_int32, []
        if ver() != ABI_VERSION:
            raise EngineError(f"{LIB_PATH} is ABI {ver()}, this module ABI {ABI_VERSION}: rebuild it")
        for name, (res, args) in SYMBOLS.items():
            fn = getattr(handle, name, None)
            if fn is None:
                raise EngineError(f"{LIB_PATH} (ABI {ABI_VERSION}) lacks {name}: rebuild it")
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def _check(rc):
    if rc != 0:
        raise EngineError(lib().mimo_last_error().decode() or f"mimo error {rc}")


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


def _ptr(a, ctype):
    return a.ctypes.data_as(ctypes.POINTER(ctype))


def as_iq(x):
    """complex array -> contiguous float64 (re, im) view."""
    x = np.ascontiguousarray(np.asarray(x, dtype=np.complex128))
    return x.view(np.float64)


class Engine:
    """One configured system (the deep-copied objects of a ``Link``) on one GPU."""

    def __init__(self, n_ant, n_sub_carr, n_fft, constel_size, cp_len, channel, receiver, tx_pos, rx_pos,
                 rx_loc_var, carrier_freqs, reroll=True, device=-1, precision=None, chan_table=None,
                 chan_replay_period=0, csi_seed=0):
        L = lib()
        self.precision = precision or default_precision()
        if self.precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(PRECISIONS)}")
        self._tx = _c(tx_pos, np.float64).reshape(-1, 3)
        self._fr = _c(carrier_freqs, np.float64)
        if self._tx.shape[0] != n_ant or self._fr.shape[0] != n_fft:
            raise ValueError("tx_pos must be [n_ant, 3] and carrier_freqs [n_fft]")
        self._tab = None
        if channel == "table":
            tab = np.asarray(chan_table, dtype=np.complex128)
            if tab.shape != (n_ant, n_fft):
                raise ValueError("chan_table must be the [n_ant, n_fft] channel matrix")
            self._tab = np.ascontiguousarray(tab).view(np.float64)
        cfg = MimoConfig(n_ant=n_ant, n_sub_carr=n_sub_carr, n_fft=n_fft, constel_size=constel_size, cp_len=cp_len,
                         channel_kind=CH_KINDS[channel], receiver_kind=RX_KINDS[receiver], device=device,
                         rx_loc_var=float(rx_loc_var), reroll_chan=int(bool(reroll)),
                         precision=PRECISIONS[self.precision],
                         tx_pos=_ptr(self._tx, ctypes.c_double), carrier_freqs=_ptr(self._fr, ctypes.c_double),
                         chan_table=_ptr(self._tab, ctypes.c_double) if self._tab is not None else None,
                         chan_replay_period=int(chan_replay_period), csi_seed=int(csi_seed))
        cfg.rx_pos[:] = [float(v) for v in rx_pos]
        h = L.mimo_engine_create(ctypes.byref(cfg))
        if not h:
            raise ValueError(L.mimo_last_error().decode())
        self._h, self._L = h, L   # the library this handle belongs to
        self.n_sub_carr, self.constel_size = n_sub_carr, constel_size

    @staticmethod
    def make_point(ibo_db, snr_db, avg_symbol_power, pa_kind, sat_pow=0.0, p_hardness=0.0, toi_coeff=0.0,
                   cnc_pa_kind=None, cnc_sat_pow=0.0, cnc_toi_coeff=0.0, cnc_alpha=1.0, csi_eps=None,
                   array_alpha=None):
        """A mimo_point from the per-point object state (Link.point_params() keys)."""
        return MimoPoint(ibo_db=float(ibo_db), snr_db=float(snr_db), avg_symbol_power=float(avg_symbol_power),
                         pa_kind=PA_KINDS[pa_kind], cnc_pa_kind=PA_KINDS[cnc_pa_kind or pa_kind],
                         sat_pow=float(sat_pow), p_hardness=float(p_hardness), toi_coeff=float(toi_coeff),
                         cnc_sat_pow=float(cnc_sat_pow), cnc_toi_coeff=float(cnc_toi_coeff),
                         cnc_alpha=float(cnc_alpha), csi_eps=-1.0 if csi_eps is None else float(csi_eps),
                         array_alpha=0.0 if array_alpha is None else float(array_alpha))

    def set_point(self, ibo_db, snr_db, avg_symbol_power, pa_kind, **kw):
        pt = self.make_point(ibo_db, snr_db, avg_symbol_power, pa_kind, **kw)
        _check(self._L.mimo_engine_set_point(self._h, ctypes.byref(pt)))

    def run_points(self, points, seeds, first_trials, n_trials, iters, incl_clean=False, per_trial=False):
        """Many grid points in as few launches as possible (mimo_engine_run_points).
        points: list of dicts (make_point keywords) or MimoPoint.  -> (err[P, n_idx],
        bits[P, n_idx], per_trial[sum n_trials, n_idx] or None)."""
        P = len(points)
        arr = (MimoPoint * max(1, P))()
        for i, pt in enumerate(points):
            arr[i] = pt if isinstance(pt, MimoPoint) else self.make_point(**pt)
        it = _c(sorted(set(int(i) for i in iters)), np.int32)
        n_idx = len(it) + (1 if incl_clean else 0)
        sd = _c(np.asarray([int(x) & 0xFFFFFFFFFFFFFFFF for x in seeds], dtype=np.uint64).reshape(-1), np.uint64)
        ft = _c(np.asarray(first_trials, dtype=np.uint64).reshape(-1), np.uint64)
        nt = _c(np.asarray(n_trials, dtype=np.uint64).reshape(-1), np.uint64)
        if not (len(sd) == len(ft) == len(nt) == P):
            raise ValueError("points, seeds, first_trials and n_trials must have the same length")
        err = np.zeros((P, n_idx), np.uint64)
        bits = np.zeros((P, n_idx), np.uint64)
        pt = np.zeros((int(nt.sum()), n_idx), np.uint32) if per_trial else None
        _check(self._L.mimo_engine_run_points(self._h, P, arr, _ptr(sd, ctypes.c_uint64), _ptr(ft, ctypes.c_uint64),
                                              _ptr(nt, ctypes.c_uint64), _ptr(it, ctypes.c_int32), len(it),
                                              int(bool(incl_clean)), _ptr(err, ctypes.c_uint64),
                                              _ptr(bits, ctypes.c_uint64),
                                              _ptr(pt, ctypes.c_uint32) if pt is not None else None))
        return err, bits, pt

    def run(self, seed, first_trial, n_trials, iters, incl_clean=False, per_trial=False):
        """-> (err[n_idx], bits[n_idx], per_trial[n_trials, n_idx] or None)."""
        it = _c(sorted(set(int(i) for i in iters)), np.int32)
        n_idx = len(it) + (1 if incl_clean else 0)
        err = np.zeros(n_idx, np.uint64)
        bits = np.zeros(n_idx, np.uint64)
        pt = np.zeros((int(n_trials), n_idx), np.uint32) if per_trial else None
        _check(self._L.mimo_engine_run(self._h, int(seed) & 0xFFFFFFFFFFFFFFFF, int(first_trial), int(n_trials),
                                     _ptr(it, ctypes.c_int32), len(it), int(bool(incl_clean)),
                                     _ptr(err, ctypes.c_uint64), _ptr(bits, ctypes.c_uint64),
                                     _ptr(pt, ctypes.c_uint32) if pt is not None else None))
        return err, bits, pt

    @property
    def kernel_ms(self):
        return self._L.mimo_engine_last_kernel_ms(self._h)

    def describe(self):
        return self._L.mimo_engine_describe(self._h).decode()

    def close(self):
        if getattr(self, "_h", None):
            self._L.mimo_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------------------ fine-seam helpers
def qam_map(constel_size, labels):
    lab = _c(labels, np.int32).reshape(-1)
    out = np.empty(lab.size, np.complex128)
    _check(lib().mimo_qam_map(int(constel_size), _ptr(lab, ctypes.c_int32), lab.size,
                              _ptr(out.view(np.float64), ctypes.c_double)))
    return out


def qam_slice(constel_size, symbols):
    z = as_iq(np.asarray(symbols).reshape(-1))
    out = np.empty(z.size // 2, np.int32)
    _check(lib().mimo_qam_slice(int(constel_size), _ptr(z, ctypes.c_double), out.size, _ptr(out, ctypes.c_int32)))
    return out.astype(np.int64)


def qam_llr(constel_size, symbols, noise_var):
    z = as_iq(np.asarray(symbols).reshape(-1))
    n = z.size // 2
    nv = _c(np.broadcast_to(np.asarray(noise_var, np.float64), (n,)), np.float64)
    nb = int(np.log2(constel_size))
    out = np.empty(n * nb, np.float64)
    _check(lib().mimo_qam_llr(int(constel_size), _ptr(z, ctypes.c_double), n, _ptr(nv, ctypes.c_double),
                              _ptr(out, ctypes.c_double)))
    return out


def fft(x, inverse=False):
    x = np.asarray(x, np.complex128)
    shape = x.shape
    xi = as_iq(x.reshape(-1, shape[-1]))
    out = np.empty(x.size, np.complex128)
    _check(lib().mimo_fft(shape[-1], x.size // shape[-1], int(inverse), _ptr(xi, ctypes.c_double),
                          _ptr(out.view(np.float64), ctypes.c_double)))
    return out.reshape(shape)


def ofdm_tx(symbols, n_fft, n_sub_carr, cp_len):
    s = np.asarray(symbols, np.complex128)
    if s.shape[-1] != n_sub_carr:
        raise ValueError("mod_symbols length must match n_sub_carr value")
    batch = s.size // n_sub_carr
    out = np.empty(batch * (n_fft + cp_len), np.complex128)
    _check(lib().mimo_ofdm_tx(n_fft, n_sub_carr, cp_len, batch, _ptr(as_iq(s), ctypes.c_double),
                              _ptr(out.view(np.float64), ctypes.c_double)))
    return out.reshape(s.shape[:-1] + (n_fft + cp_len,))


def ofdm_rx(td, n_fft, n_sub_carr, cp_len):
    t = np.asarray(td, np.complex128)
    batch = t.size // (n_fft + cp_len)
    out = np.empty(batch * n_sub_carr, np.complex128)
    _check(lib().mimo_ofdm_rx(n_fft, n_sub_carr, cp_len, batch, _ptr(as_iq(t), ctypes.c_double),
                              _ptr(out.view(np.float64), ctypes.c_double)))
    return out.reshape(t.shape[:-1] + (n_sub_carr,))


def pa(kind, x, sat_pow=0.0, p_hardness=0.0, toi_coeff=0.0):
    xa = np.asarray(x)
    is_real = not np.iscomplexobj(xa)
    x2 = np.asarray(xa, np.complex128)
    out = np.empty(x2.size, np.complex128)
    _check(lib().mimo_pa(PA_KINDS[kind], float(sat_pow), float(p_hardness), float(toi_coeff),
                         _ptr(as_iq(x2.reshape(-1)), ctypes.c_double), x2.size,
                         _ptr(out.view(np.float64), ctypes.c_double)))
    out = out.reshape(x2.shape)
    return out.real.copy() if is_real else out


def calc_alpha(ibo_db):
    """Bussgang gain per IBO [dB] by the float64 kernels' segment table (alpha_fit.h)."""
    ibo = np.ascontiguousarray(np.atleast_1d(np.asarray(ibo_db, np.float64)))
    out = np.empty(ibo.size, np.float64)
    _check(lib().mimo_calc_alpha(_ptr(ibo, ctypes.c_double), ibo.size, _ptr(out, ctypes.c_double)))
    return out.reshape(np.shape(ibo_db))


def mrt_precode(h_sc):
    h = np.asarray(h_sc, np.complex128)
    A, K = h.shape
    out = np.empty(A * K, np.complex128)
    _check(lib().mimo_mrt_precode(A, K, _ptr(as_iq(h), ctypes.c_double), _ptr(out.view(np.float64), ctypes.c_double)))
    return out.reshape(A, K)


def combine(h, y):
    h = np.asarray(h, np.complex128)
    y = np.asarray(y, np.complex128)
    A, K = h.shape
    out = np.empty(K, np.complex128)
    _check(lib().mimo_combine(A, K, _ptr(as_iq(h), ctypes.c_double), _ptr(as_iq(y), ctypes.c_double),
                              _ptr(out.view(np.float64), ctypes.c_double)))
    return out


def awgn(x, noise_std, seed, counter):
    xa = np.asarray(x, np.complex128)
    out = np.empty(xa.size, np.complex128)
    _check(lib().mimo_awgn(int(seed) & 0xFFFFFFFFFFFFFFFF, int(counter), xa.size, float(noise_std),
                           _ptr(as_iq(xa.reshape(-1)), ctypes.c_double), _ptr(out.view(np.float64), ctypes.c_double)))
    return out.reshape(xa.shape)


def count_bit_errors(a, b):
    a = _c(a, np.int64).reshape(-1)
    b = _c(b, np.int64).reshape(-1)
    out = np.zeros(1, np.int64)
    _check(lib().mimo_count_bit_errors(_ptr(a, ctypes.c_int64), _ptr(b, ctypes.c_int64), a.size,
                                       _ptr(out, ctypes.c_int64)))
    return int(out[0])


def cnc_receive(constel_size, n_fft, pa_kind, sat_pow, p_hardness, toi_coeff, alpha, iters, rx_sc, return_bits=True):
    """{iteration: detected labels}, or with ``return_bits=False`` {iteration: the corrected
    slicer input rx - d} (mimo_cnc_receive_ex)."""
    z = as_iq(np.asarray(rx_sc).reshape(-1))
    S = z.size // 2
    it = _c(sorted(set(int(i) for i in iters)), np.int32)
    lab = np.empty((len(it), S), np.int32) if return_bits else None
    cor = None if return_bits else np.empty((len(it), S), np.complex128)
    _check(lib().mimo_cnc_receive_ex(int(constel_size), int(n_fft), S, PA_KINDS[pa_kind], float(sat_pow),
                                     float(p_hardness), float(toi_coeff), float(alpha), _ptr(it, ctypes.c_int32),
                                     len(it), _ptr(z, ctypes.c_double),
                                     _ptr(lab, ctypes.c_int32) if lab is not None else None,
                                     _ptr(cor.view(np.float64), ctypes.c_double) if cor is not None else None))
    if return_bits:
        return {int(i): lab[j].astype(np.int64) for j, i in enumerate(it)}
    return {int(i): cor[j] for j, i in enumerate(it)}
