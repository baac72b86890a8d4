"""CPU check of pass 1's polar form for Rayleigh channels with CSI error (csrc/trial_kernel.h
CSI_POLAR, mp_model.py:264-282 restated): with h = rho_h e^{j phi_h} and z = rho_z e^{j phi_z}
drawn from (radius word, angle word) pairs as Box-Muller does (philox.h box_muller: angle =
2 pi w1 2^-32), the estimate Hhat = a h + sc z has

    |Hhat|^2       = a^2 rho_h^2 + sc^2 rho_z^2 + 2 a sc rho_h rho_z cos(phi_h - phi_z)
    h conj(Hhat)   = a rho_h^2 + sc rho_h rho_z e^{j (phi_h - phi_z)}

and the angle difference is the 32-bit word difference modulo 2^32 (exact).  The GPU parity
cases pin the kernel (tests/test_gpu_sizes.py CSI rows); this pins the algebra."""
import numpy as np


def test_polar_identities_match_cartesian():
    rng = np.random.default_rng(11)
    n = 20000
    w0h, w1h, w0z, w1z = (rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32) for _ in range(4))
    fr = rng.uniform(0.9, 1.1, n)  # the FSPL ratio the kernel folds into rho_h
    r2h = -np.log((w0h.astype(np.float64) + 0.5) * 2.0 ** -32) * fr ** 2
    r2z = -np.log((w0z.astype(np.float64) + 0.5) * 2.0 ** -32)
    h = np.sqrt(r2h) * np.exp(2j * np.pi * w1h.astype(np.float64) * 2.0 ** -32)
    z = np.sqrt(r2z) * np.exp(2j * np.pi * w1z.astype(np.float64) * 2.0 ** -32)
    for a, sc in ((np.sqrt(1 - 0.1 ** 2), 0.1 * 1.3), (np.sqrt(1 - 0.4 ** 2), 0.4 * 0.7)):
        hhat = a * h + sc * z
        dw = (w1h - w1z).astype(np.uint32)  # wraps modulo 2^32 like the kernel's uint32 difference
        d = 2 * np.pi * dw.astype(np.float64) * 2.0 ** -32
        rhz = np.sqrt(r2h * r2z)
        e2 = a * a * r2h + sc * sc * r2z + 2 * a * sc * rhz * np.cos(d)
        cc = a * r2h + sc * rhz * np.exp(1j * d)
        np.testing.assert_allclose(e2, np.abs(hhat) ** 2, rtol=1e-11, atol=1e-13)
        np.testing.assert_allclose(cc, h * np.conj(hhat), rtol=1e-11, atol=1e-13)
