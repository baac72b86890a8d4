"""CPU check of the FFT's twiddle-absorbing butterflies (csrc/team_fft.h bfly_ct, dft8_ct,
dft16_ct; round 5): the butterfly network, restated here operation by operation in NumPy,
equals "multiply input r by z^r, then the radix-R DFT" (y[k] = sum_r W^(r k) z^r v[r], W =
exp(DIR j 2 pi / R), z conjugated for the inverse) for both directions and twiddles all
round the circle -- including the angles where cos is 6e-17 (the cot-tan form's edge).
The GPU parity tests pin the kernels themselves; this pins the algebra and the constant
rows (ct_rev) the host table builds."""
import numpy as np
import pytest


def ct_rev(R, ns, jm, q):
    """team_fft.h ct_rev: rows of a radix-R stage, angles in revolutions."""
    th = -jm / (R * ns)
    if R == 8:
        return [4 * th, 2 * th, th, th - 0.125][q]
    return [8 * th, 4 * th, 2 * th, 2 * th - 0.125, th, th - 0.0625, th - 0.125, th - 0.1875][q]


def ct_const(rev):
    a = 2 * np.pi * rev
    c = np.cos(a)
    return c, np.sin(a) / c


def bfly_ct(DIR, ROT, a, b, ct):
    c, t = ct
    tt = t if DIR < 0 else -t
    ux = b.real - tt * b.imag
    uy = b.imag + tt * b.real
    if not ROT:
        return complex(a.real + c * ux, a.imag + c * uy), complex(a.real - c * ux, a.imag - c * uy)
    cd = -c if DIR < 0 else c
    return complex(a.real - cd * uy, a.imag + cd * ux), complex(a.real + cd * uy, a.imag - cd * ux)


def dft8_ct(DIR, v, zc):
    v = list(v)
    a0, a1 = [0j] * 4, [0j] * 4
    for r in range(4):
        a0[r], a1[r] = bfly_ct(DIR, False, v[r], v[r + 4], zc[0])
    b = [[0j] * 4 for _ in range(2)]
    for r0 in range(2):
        b[r0][0], b[r0][2] = bfly_ct(DIR, False, a0[r0], a0[r0 + 2], zc[1])
        b[r0][1], b[r0][3] = bfly_ct(DIR, True, a1[r0], a1[r0 + 2], zc[1])
    out = [0j] * 8
    out[0], out[4] = bfly_ct(DIR, False, b[0][0], b[1][0], zc[2])
    out[1], out[5] = bfly_ct(DIR, False, b[0][1], b[1][1], zc[3])
    out[2], out[6] = bfly_ct(DIR, True, b[0][2], b[1][2], zc[2])
    out[3], out[7] = bfly_ct(DIR, True, b[0][3], b[1][3], zc[3])
    return np.array(out)


def dft16_ct(DIR, v, zc):
    v = list(v)
    a = [[0j] * 8 for _ in range(2)]
    for r in range(8):
        a[0][r], a[1][r] = bfly_ct(DIR, False, v[r], v[r + 8], zc[0])
    b = [[0j] * 4 for _ in range(4)]
    for r in range(4):
        b[r][0], b[r][2] = bfly_ct(DIR, False, a[0][r], a[0][r + 4], zc[1])
        b[r][1], b[r][3] = bfly_ct(DIR, True, a[1][r], a[1][r + 4], zc[1])
    c = [[0j] * 8 for _ in range(2)]
    for r0 in range(2):
        c[r0][0], c[r0][4] = bfly_ct(DIR, False, b[r0][0], b[r0 + 2][0], zc[2])
        c[r0][1], c[r0][5] = bfly_ct(DIR, False, b[r0][1], b[r0 + 2][1], zc[3])
        c[r0][2], c[r0][6] = bfly_ct(DIR, True, b[r0][2], b[r0 + 2][2], zc[2])
        c[r0][3], c[r0][7] = bfly_ct(DIR, True, b[r0][3], b[r0 + 2][3], zc[3])
    out = [0j] * 16
    for m in range(4):
        out[m], out[m + 8] = bfly_ct(DIR, False, c[0][m], c[1][m], zc[4 + m])
        out[m + 4], out[m + 12] = bfly_ct(DIR, True, c[0][m + 4], c[1][m + 4], zc[4 + m])
    return np.array(out)


@pytest.mark.parametrize("R", [8, 16])
@pytest.mark.parametrize("DIR", [-1, +1])
@pytest.mark.parametrize("ns", [1, 8, 16, 64])
def test_absorbed_twiddle_dft_equals_twiddle_then_dft(R, DIR, ns):
    rng = np.random.default_rng(R * 100 + ns + (DIR > 0))
    k = np.arange(R)
    W = np.exp(DIR * 2j * np.pi * np.outer(k, k) / R)
    worst = 0.0
    for jm in range(ns):
        z = np.exp(-2j * np.pi * jm / (R * ns))  # forward twiddle base (team_fft.h)
        zd = z if DIR < 0 else np.conj(z)
        zc = [ct_const(ct_rev(R, ns, jm, q)) for q in range(4 if R == 8 else 8)]
        for _ in range(3):
            v = rng.standard_normal(R) + 1j * rng.standard_normal(R)
            want = W @ (zd ** k * v)
            got = dft8_ct(DIR, v, zc) if R == 8 else dft16_ct(DIR, v, zc)
            worst = max(worst, float(np.max(np.abs(got - want)) / np.max(np.abs(want))))
    assert worst < 1e-14, worst


def test_cot_tan_constants_stay_finite_at_quarter_turns():
    """cos of a quarter turn is 6.1e-17 in double, never 0: tan is ~1.6e16, finite, and
    c * tan rounds back to sin (what bfly_ct relies on)."""
    for rev in (-0.25, 0.25, -0.75, -0.5 + 0.25):
        c, t = ct_const(rev)
        assert c != 0.0 and np.isfinite(t)
        assert abs(c * t - np.sin(2 * np.pi * rev)) < 1e-15
