"""CPU model of the split FFT (csrc/split_fft.h; the fp64 F 8192 instance): one 512-thread
team, 16 points per thread, each transform as two 4096-point sub-transforms (one per lane
half of every wave) plus a radix-2 stage whose operands meet through v_permlane32_swap
instead of an LDS exchange.  Restated here lane by lane in NumPy -- the thread -> (group,
virtual thread) map, the frequency layout (bin tau + T m at freq thread tau = 2 vt + g), the
half-wave swap semantics (lanes 32-63 of vdst <-> lanes 0-31 of src) and the cot-tan radix-2
butterflies with the host table's constants -- and checked against numpy.fft for both
directions, including the inverse -> forward round trip the kernel runs per antenna."""
import numpy as np
import pytest

F, T = 8192, 512
P, H, TH = F // T, F // 2, T // 2


def vthread(t):
    return ((t >> 6) << 5) | (t & 31)


def group(t):
    return (t >> 5) & 1


def freq_thread(t):
    return (vthread(t) << 1) | group(t)


def swap_halves(a, b):
    """v_permlane32_swap(vdst=a, src=b) on per-thread arrays [T] (64-lane waves)."""
    a, b = a.copy(), b.copy()
    for w in range(T // 64):
        lo, hi = slice(64 * w, 64 * w + 32), slice(64 * w + 32, 64 * w + 64)
        a_hi = a[hi].copy()
        a[hi] = b[lo]
        b[lo] = a_hi
    return a, b


def r2_table():
    """(cos, tan) of exp(-j 2 pi n / F), n < F / 2 (engine.hip split table)."""
    ang = -2 * np.pi * np.arange(H) / F
    return np.cos(ang), np.sin(ang) / np.cos(ang)


def bfly_ct(DIR, a, b, c, t):
    """team_fft.h bfly_ct<DIR, false>: a + z b, a - z b with z = c (1 + j tt)."""
    tt = t if DIR < 0 else -t
    ux = b.real - tt * b.imag
    uy = b.imag + tt * b.real
    return a + c * (ux + 1j * uy), a - c * (ux + 1j * uy)


def sub_dft(d, DIR):
    """Each group's 4096-point transform in the sub cyclic layout (vt, m): element vt + TH m."""
    out = np.empty_like(d)
    t = np.arange(T)
    for g in (0, 1):
        sel = t[group(t) == g]
        vt = vthread(sel)
        x = np.empty(H, complex)
        for m in range(P):
            x[vt + TH * m] = d[sel, m]
        y = np.fft.ifft(x) * H if DIR > 0 else np.fft.fft(x)
        for m in range(P):
            out[sel, m] = y[vt + TH * m]
    return out


def inverse(d):
    c, tn = r2_table()
    d = sub_dft(d, +1)
    t = np.arange(T)
    for m in range(P // 2):
        d[:, m], d[:, m + P // 2] = swap_halves(d[:, m], d[:, m + P // 2])
    for m in range(P // 2):
        n = vthread(t) + TH * (m + (P // 2) * group(t))
        d[:, m], d[:, m + P // 2] = bfly_ct(+1, d[:, m], d[:, m + P // 2], c[n], tn[n])
    return d


def forward(d):
    c, tn = r2_table()
    t = np.arange(T)
    d = d.copy()
    for m in range(P // 2):
        n = vthread(t) + TH * (m + (P // 2) * group(t))
        a, b = d[:, m], d[:, m + P // 2]
        u = a - b
        d[:, m] = a + b
        d[:, m + P // 2] = c[n] * ((u.real - tn[n] * u.imag) + 1j * (u.imag + tn[n] * u.real))
    for m in range(P // 2):
        d[:, m], d[:, m + P // 2] = swap_halves(d[:, m], d[:, m + P // 2])
    return sub_dft(d, -1)


def time_index():
    """[T, P] time sample held at (thread, register) after inverse()."""
    t = np.arange(T)
    n = np.empty((T, P), np.int64)
    for m in range(P // 2):
        base = vthread(t) + TH * (m + (P // 2) * group(t))
        n[:, m], n[:, m + P // 2] = base, base + H
    return n


def test_freq_thread_is_a_permutation_with_thread0_fixed():
    tau = freq_thread(np.arange(T))
    assert sorted(tau) == list(range(T)) and tau[0] == 0


def test_inverse_matches_numpy():
    rng = np.random.default_rng(1)
    X = rng.standard_normal(F) + 1j * rng.standard_normal(F)
    tau = freq_thread(np.arange(T))
    d = np.stack([X[tau + T * m] for m in range(P)], axis=1)
    x = inverse(d)
    want = np.fft.ifft(X) * F
    n = time_index()
    assert sorted(n.ravel()) == list(range(F))
    assert np.max(np.abs(x - want[n])) < 1e-11 * np.max(np.abs(want))


def test_forward_matches_numpy():
    rng = np.random.default_rng(2)
    x = rng.standard_normal(F) + 1j * rng.standard_normal(F)
    n = time_index()
    X = forward(x[n])
    want = np.fft.fft(x)
    tau = freq_thread(np.arange(T))
    got = np.empty(F, complex)
    for m in range(P):
        got[tau + T * m] = X[:, m]
    assert np.max(np.abs(got - want)) < 1e-11 * np.max(np.abs(want))


@pytest.mark.parametrize("clip", [False, True])
def test_round_trip_with_pointwise_step(clip):
    """inverse -> pointwise map on the time layout -> forward == the same chain in NumPy."""
    rng = np.random.default_rng(3)
    X = rng.standard_normal(F) + 1j * rng.standard_normal(F)
    tau = freq_thread(np.arange(T))
    d = np.stack([X[tau + T * m] for m in range(P)], axis=1)
    x = inverse(d)
    if clip:
        x = x * np.minimum(1.0, 40.0 / np.maximum(np.abs(x), 1e-300))
    Y = forward(x)
    xr = np.fft.ifft(X) * F
    if clip:
        xr = xr * np.minimum(1.0, 40.0 / np.maximum(np.abs(xr), 1e-300))
    want = np.fft.fft(xr)
    got = np.empty(F, complex)
    for m in range(P):
        got[tau + T * m] = Y[:, m]
    assert np.max(np.abs(got - want)) < 1e-10 * np.max(np.abs(want))


def test_r2_twiddle_product_form_near_quarter_turn():
    """The (cos a, tan a) form at a = -pi/2 (n = F/4: cos 6.1e-17, tan -1.6e16) and its
    neighbours: c (u.x - t u.y) + j c (u.y + t u.x) equals e^{ja} u to a few ulp of |u|, in
    both directions -- c t rounds to sin a, so the large tangent loses nothing."""
    c, t = r2_table()
    rng = np.random.default_rng(4)
    for n in (F // 4 - 2, F // 4 - 1, F // 4, F // 4 + 1, F // 4 + 2, 0, H - 1):
        for DIR in (-1, +1):
            u = complex(rng.standard_normal(), rng.standard_normal())
            zero = np.zeros(1, complex)
            got = bfly_ct(DIR, zero, np.array([u]), c[n], t[n])[0][0]
            want = np.exp(DIR * 2j * np.pi * n / F) * u
            assert abs(got - want) <= 4e-16 * abs(u), (n, DIR, abs(got - want) / abs(u))
