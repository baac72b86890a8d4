"""Philox4x32-10 counter-based RNG and the engine's random-stream layout (NumPy, CPU).

TEST INFRASTRUCTURE ONLY.  Nothing in the product imports this module; only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg use it,
as the checker.

The reference draws its randomness from NumPy PCG64 streams
(``mp_model.py:121-125``: ``bit_rng``, ``my_noise.rng_gen``, ``loc_rng``;
``channel.py:209-212,262-275``: Rayleigh ``rng_gen``).  PCG64 + ziggurat normals are
sequential and cannot be replayed per element on a GPU, so the engine replaces them with
Philox4x32-10 (Salmon et al., SC'11, "Parallel random numbers: as easy as 1, 2, 3")
keyed by the 64-bit run seed and addressed by (element, trial, stream, aux).  This file
is the single CPU statement of that layout; ``csrc/philox.h`` is the device statement.
Parity with the reference is obtained by *injecting these draws into the reference*
(``tests/golden/make_golden.py``), so both sides see identical random inputs.

Stream layout (counter words c0..c3, key = (seed_lo32, seed_hi32)):

=========  ==========================  =========================================
stream id  counter                      use
=========  ==========================  =========================================
1 BITS     (k >> 2, trial, 1, 0)        word[k & 3] & (M-1) = QAM label of subcarrier k
2 CHAN     (q, trial, 2, a)             2 CN(0,1) draws for antenna a, sub-carrier pair q
3 NOISE    (q, trial, 3, 0)             2 CN(0,1) AWGN draws for sub-carrier pair q
4 CSI      (q, trial, 4, a)             2 CN(0,1) CSI-error draws (mp_model.py:264-288)
5 LOC      (0, trial, 5, 0)             RX position jitter, 2 uniforms (mp_model.py:190-201)
=========  ==========================  =========================================

Sub-carrier pairing ("quarter pairing"): with Q = S/4, sub-carrier k lives in half
h = k // (S/2) at offset r = k % (S/2); its pair index is q = h*Q + r % Q and its slot in
the pair is r // Q.  Pair q covers k1 = (q // Q)*(S/2) + q % Q and k2 = k1 + Q.  (On the
GPU, k1 and k2 land in the same thread whenever Q is a multiple of the team size.)

Complex normal from two words (w0, w1):  u1 = (w0 + 0.5) 2^-32, u2 = w1 2^-32,
z = sqrt(-ln u1) * exp(j 2 pi u2)   ->  E|z|^2 = 1  (Box-Muller).
"""
from __future__ import annotations

import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint64(0x9E3779B9)
W1 = np.uint64(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)
S32 = np.uint64(32)

STREAM_BITS = 1
STREAM_CHAN = 2
STREAM_NOISE = 3
STREAM_CSI = 4
STREAM_LOC = 5


def philox4x32_10(c0, c1, c2, c3, key):
    """Philox4x32 with 10 rounds; counters broadcast, ``key`` is a 64-bit int.

    Returns four uint32 arrays.  Known-answer vectors: ``tests/test_oracle_philox.py``.
    """
    k0 = np.uint64(int(key) & 0xFFFFFFFF)
    k1 = np.uint64((int(key) >> 32) & 0xFFFFFFFF)
    c0, c1, c2, c3 = np.broadcast_arrays(*(np.asarray(c, dtype=np.uint64) for c in (c0, c1, c2, c3)))
    c0, c1, c2, c3 = (c & MASK for c in (c0, c1, c2, c3))
    for r in range(10):
        if r:
            k0 = (k0 + W0) & MASK
            k1 = (k1 + W1) & MASK
        p0 = M0 * c0
        p1 = M1 * c2
        c0, c1, c2, c3 = ((p1 >> S32) ^ c1 ^ k0, p1 & MASK, (p0 >> S32) ^ c3 ^ k1, p0 & MASK)
    return tuple(c.astype(np.uint32) for c in (c0, c1, c2, c3))


def box_muller(w0, w1):
    """Two uint32 words -> one CN(0,1) sample (float64)."""
    u1 = (w0.astype(np.float64) + 0.5) * 2.0 ** -32
    u2 = w1.astype(np.float64) * 2.0 ** -32
    rho = np.sqrt(-np.log(u1))
    ang = 2.0 * np.pi * u2
    return rho * np.cos(ang) + 1j * rho * np.sin(ang)


def pair_index(k, n_sc):
    """Quarter pairing: sub-carrier index -> (pair q, slot 0/1)."""
    k = np.asarray(k, dtype=np.int64)
    half, quarter = n_sc // 2, n_sc // 4
    h, r = k // half, k % half
    return h * quarter + r % quarter, r // quarter


def _check_sc(n_sc):
    if n_sc % 4:
        raise ValueError("the engine requires n_sub_carr % 4 == 0 (sub-carrier pairing)")


def qam_labels(seed, trials, n_sc, constel_size, user=0):
    """[T, S] int64 QAM labels (stream BITS; aux = user index for multi-user runs)."""
    trials = np.asarray(trials, dtype=np.uint64).reshape(-1, 1)
    k = np.arange(n_sc, dtype=np.uint64).reshape(1, -1)
    w = philox4x32_10(k >> np.uint64(2), trials, STREAM_BITS, int(user), seed)
    sel = (k & np.uint64(3)).astype(np.int64)
    words = np.stack(w, axis=-1)  # [T, S, 4]
    word = np.take_along_axis(words, np.broadcast_to(sel, words.shape[:2])[..., None], axis=-1)[..., 0]
    return (word & np.uint32(constel_size - 1)).astype(np.int64)


def _cn_pairs(seed, trials, n_sc, stream, aux):
    """CN(0,1) draws [T, len(aux), S] for one stream; aux = antenna indices (or [0])."""
    _check_sc(n_sc)
    trials = np.asarray(trials, dtype=np.uint64).reshape(-1, 1, 1)
    aux = np.asarray(aux, dtype=np.uint64).reshape(1, -1, 1)
    q = np.arange(n_sc // 2, dtype=np.uint64).reshape(1, 1, -1)
    w0, w1, w2, w3 = philox4x32_10(q, trials, stream, aux, seed)
    z1 = box_muller(w0, w1)
    z2 = box_muller(w2, w3)
    half, quarter = n_sc // 2, n_sc // 4
    qi = np.arange(n_sc // 2)
    k1 = (qi // quarter) * half + qi % quarter
    out = np.empty(z1.shape[:2] + (n_sc,), dtype=np.complex128)
    out[..., k1] = z1
    out[..., k1 + quarter] = z2
    return out


def chan_normals(seed, trials, n_sc, n_ant):
    """[T, A, S] CN(0,1) channel draws (stream CHAN)."""
    return _cn_pairs(seed, trials, n_sc, STREAM_CHAN, np.arange(n_ant))


def noise_normals(seed, trials, n_sc):
    """[T, S] CN(0,1) AWGN draws (stream NOISE)."""
    return _cn_pairs(seed, trials, n_sc, STREAM_NOISE, [0])[:, 0, :]


def csi_normals(seed, trials, n_sc, n_ant):
    """[T, A, S] CN(0,1) CSI-error draws (stream CSI)."""
    return _cn_pairs(seed, trials, n_sc, STREAM_CSI, np.arange(n_ant))


def loc_uniforms(seed, trials):
    """[T, 2] uniforms in [0, 1) for the RX position jitter (stream LOC)."""
    trials = np.asarray(trials, dtype=np.uint64)
    w0, w1, _, _ = philox4x32_10(0, trials, STREAM_LOC, 0, seed)
    return np.stack([w0.astype(np.float64) * 2.0 ** -32, w1.astype(np.float64) * 2.0 ** -32], axis=-1)
