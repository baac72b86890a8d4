// Bussgang gain of the soft limiter over its whole domain, for float64 kernels.
//
// Modem.calc_alpha (modulation.py:178-189): alpha(g) = 1 - e^{-g^2} + (sqrt(pi)/2) g erfc(g),
// g = 10^(IBO/20); the trial kernel evaluates it per antenna at g^2 = 10^(IBO_a/10)
// (mp_model.py:312-317).  Its per-point Horner fit covers the antennas' usual range; this
// table covers everything else without the library exp / erfc, whose f64 constants the
// compiler hoisted out of the antenna loop and spilled once per trial.
//
// Segments k = 0 .. kAlphaSegs - 1 of g in [0, 6.5), width 1/2: degree-kAlphaDeg Horner in
// u = 4 g - 2 k - 1 (in [-1, 1)) from the long-double Chebyshev interpolant at 64 nodes,
// converted to monomials.  Segment 0 holds alpha(g) / g (relative accuracy as g -> 0; the
// kernel multiplies by g).  From g = 6.5 on alpha rounds to 1 (1 - alpha ~ e^{-g^2} / 2 <
// 2^-54 from g ~ 6.1).  Measured in mpmath at 40 digits: <= 1.6e-16 relative on every
// segment (tests/test_gpu_fine_seams.py::test_calc_alpha_vs_mpmath through mimo_calc_alpha).
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <vector>

namespace mimo {

constexpr int kAlphaSegs = 13, kAlphaDeg = 16, kAlphaStride = kAlphaDeg + 1;
constexpr int kAlphaTabDoubles = kAlphaSegs * kAlphaStride;

// Host: the segment table, kAlphaTabDoubles doubles.
inline std::vector<double> alpha_segment_table() {
  std::vector<double> tab(kAlphaTabDoubles);
  constexpr int N = 64, D = kAlphaDeg;
  const long double pi = 3.14159265358979323846264338327950288L;
  const long double sqpi2 = 0.886226925452758013649083741671L;  // sqrt(pi) / 2
  for (int k = 0; k < kAlphaSegs; ++k) {
    const long double c = 0.5L * k + 0.25L, h = 0.25L;
    long double ck[D + 1];
    for (int j = 0; j <= D; ++j) {
      long double s = 0.0L;
      for (int i = 0; i < N; ++i) {
        const long double th = pi * (i + 0.5L) / N;
        const long double g = c + h * std::cos(th);
        // segment 0: alpha / g = -expm1(-g^2) / g + sqrt(pi)/2 erfc(g)
        const long double f = k == 0 ? -std::expm1(-g * g) / g + sqpi2 * std::erfc(g)
                                     : 1.0L - std::exp(-g * g) + sqpi2 * g * std::erfc(g);
        s += f * std::cos(j * th);
      }
      ck[j] = s * (j == 0 ? 1.0L : 2.0L) / N;
    }
    // Chebyshev -> monomials in u (T_{j+1} = 2 u T_j - T_{j-1})
    long double Tm1[D + 1] = {0}, T0[D + 1] = {0}, mono[D + 1] = {0};
    T0[0] = 1.0L;
    for (int j = 0; j <= D; ++j) {
      for (int i = 0; i <= D; ++i) mono[i] += ck[j] * T0[i];
      long double Tn[D + 1] = {0};
      for (int i = 0; i <= D; ++i) {
        if (i > 0) Tn[i] += (j == 0 ? 1.0L : 2.0L) * T0[i - 1];
        Tn[i] -= Tm1[i];
      }
      for (int i = 0; i <= D; ++i) {
        Tm1[i] = T0[i];
        T0[i] = Tn[i];
      }
    }
    for (int i = 0; i <= D; ++i) tab[k * kAlphaStride + i] = (double)mono[i];
  }
  return tab;
}

// Device: alpha from g^2 >= 0 (+inf allowed).  Callers pass a team-uniform g^2, so the
// segment index is uniform: the coefficients are scalar loads and SGPR operands of the
// FMAs (inline v_fma_f64: plain fma() would copy each coefficient into VGPRs first).
__device__ __forceinline__ double alpha_seg(double g2, const double* tab) {
  const double g = __builtin_sqrt(g2);
  if (!(g < 6.5)) return 1.0;
  const int k = __builtin_amdgcn_readfirstlane((int)(2.0 * g));
  const double u = fma(4.0, g, -(double)(2 * k + 1));
  using CD = const __attribute__((address_space(4))) double;
  CD* c = (CD*)tab + k * kAlphaStride;
  double acc = c[kAlphaDeg];
#pragma unroll
  for (int i = kAlphaDeg - 1; i >= 0; --i) {
    const double ci = c[i];
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(acc) : "v"(acc), "v"(u), "s"(ci));
  }
  return k == 0 ? acc * g : acc;
}

}  // namespace mimo
