// Precision traits of the fused trial kernel: one source, two arithmetic types.
//
// R = double is the reference's own precision (complex128 / float64 end to end,
// modulation.py:270, noise.py:66); R = float is the fast variant.  Everything on the
// signal chain (FFT, precoding, PA, channel, AGC, receiver) runs in R; the float
// instances keep the hardware approximations (v_rsq / v_log / v_sin ...) that the
// fp32 kernel was tuned with, the double instances use the full-precision software
// forms below (gfx950 has no f64 transcendental instructions besides rcp / rsq / sqrt
// seeds).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mimo {

template <typename R>
struct CxT;
template <>
struct CxT<float> {
  using type = float2;
};
template <>
struct CxT<double> {
  using type = double2;
};
template <typename R>
using cx = typename CxT<R>::type;
template <class C>
struct RealOf;
template <>
struct RealOf<float2> {
  using type = float;
};
template <>
struct RealOf<double2> {
  using type = double;
};
template <class C>
using real_of = typename RealOf<C>::type;

__device__ __forceinline__ float2 mkc(float a, float b) { return make_float2(a, b); }
__device__ __forceinline__ double2 mkc(double a, double b) { return make_double2(a, b); }
template <typename R>
__device__ __forceinline__ cx<R> czero() {
  return mkc(R(0), R(0));
}
__device__ __forceinline__ float fmar(float a, float b, float c) { return fmaf(a, b, c); }
__device__ __forceinline__ double fmar(double a, double b, double c) { return fma(a, b, c); }
__device__ __forceinline__ float minr(float a, float b) { return fminf(a, b); }
__device__ __forceinline__ double minr(double a, double b) { return fmin(a, b); }
__device__ __forceinline__ float absr(float a) { return fabsf(a); }
__device__ __forceinline__ float floor_r(float a) { return floorf(a); }
__device__ __forceinline__ double floor_r(double a) { return floor(a); }
__device__ __forceinline__ double absr(double a) { return fabs(a); }

// ---------------------------------------------------------------- fp32: hardware forms
__device__ __forceinline__ float rsq_r(float x) { return __builtin_amdgcn_rsqf(x); }   // rsq(0) = inf
__device__ __forceinline__ float sqrt_r(float x) { return __builtin_amdgcn_sqrtf(x); }  // raw v_sqrt (1 ulp)
__device__ __forceinline__ float log2_r(float x) { return __builtin_amdgcn_logf(x); }
__device__ __forceinline__ float exp2_r(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float rcp_r(float x) { return 1.0f / x; }
__device__ __forceinline__ float sqrt_ieee(float x) { return __builtin_sqrtf(x); }  // correctly rounded

// ---------------------------------------------------------------- fp64: software forms
// 1/sqrt(x) for finite x > 0: v_rsq_f64 seed + two Newton steps.  (Callers select away
// the result for x = 0, where the fp32 form returns inf.)
__device__ __forceinline__ double rsq_r(double x) {
  double y = __builtin_amdgcn_rsq(x);
  const double h = 0.5 * x;
#pragma unroll
  for (int i = 0; i < 2; ++i) y = fma(y, fma(-h * y, y, 0.5), y);
  return y;
}
__device__ __forceinline__ double sqrt_r(double x) { return __builtin_sqrt(x); }
__device__ __forceinline__ double sqrt_ieee(double x) { return __builtin_sqrt(x); }
__device__ __forceinline__ double log2_r(double x) { return log2(x); }
__device__ __forceinline__ double exp2_r(double x) { return exp2(x); }
__device__ __forceinline__ double rcp_r(double x) { return 1.0 / x; }

// ---------------------------------------------------------------- fp64: table-driven forms
// The fp64 trial kernel's Box-Muller draws (2 A S normals per trial) dominate its
// transcendental work, so they use LDS tables instead of the long series above
// (ln: ~13 f64 ops instead of ~25 plus a Newton reciprocal for the atanh series; sincos:
// ~15 instead of ~35 for a quadrant Taylor series; the series forms are in git history).
// Table (host-built, engine.hip lut64_table, loaded into LDS at kernel start):
//   [0, 512):   (c_i, -ln c_i) for m in bucket i of [0.5, 1) (ln_unit: the top 9 mantissa
//               bits); c_i ~ 1/centre_i rounded to 12 bits, c_i = 1 for the top bucket
//   [512, 768): (cos, sin)(2 pi i / 256)
constexpr int kLnTab = 512, kScTab = 256, kLut64 = kLnTab + kScTab;
static __shared__ double2 lut64[kLut64];
// Diagnostic builds only (-DMIMO_DIAG_LUT_SEQ, wrong results): the table index's low 4 bits
// replaced by the lane's, so every ds_read_b128 lane group (16 lanes with distinct lane & 15,
// MI355X_MICROARCH §LDS) reads 16 distinct bank quads -- the random-index reads' bank
// conflicts removed, their count and addresses' dependence kept (the conflict attribution
// of profiles/r06/lut/).
#ifdef MIMO_DIAG_LUT_SEQ
__device__ __forceinline__ uint32_t lut_idx(uint32_t i) { return (i & ~15u) | (threadIdx.x & 15u); }
#else
__device__ __forceinline__ uint32_t lut_idx(uint32_t i) { return i; }
#endif

// sin / cos of 2 pi w 2^-32 (w: a uint32 word, revolutions): i = nearest 256th,
// phi = 2 pi (w - i 2^24) 2^-32 in [-pi/256, pi/256], series to phi^7 / phi^6 and the
// angle sum with the table's (cos, sin)(2 pi i / 256).  <= ~1.5 ulp.
// The series run in the integer residual f itself (coefficients scaled by powers of
// h = 2 pi 2^-32): sin = f (h - h^3 f^2 / 6 + ...), cos = 1 - h^2 f^2 / 2 + ... -- one
// multiply fewer than forming phi = h f first.
__device__ __forceinline__ void sincos_lut(uint32_t w, double& sn, double& cs) {
  const uint32_t i = (w + 0x800000u) >> 24;  // wraps to 0 near a full revolution
  // w - i 2^24 = the low 24 bits of w sign-extended (one v_bfe_i32), in [-2^23, 2^23)
  const double f = (double)(((int)(w << 8)) >> 8);
  constexpr double h = 1.4629180792671596e-09;    // 2 pi 2^-32
  constexpr double h2 = h * h;
  const double z = f * f;                         // exact (< 2^46)
  double ps = fma(z, -(h2 * h2 * h2 * h) / 5040, (h2 * h2 * h) / 120);
  ps = fma(ps, z, -(h2 * h) / 6);
  ps = fma(ps, z, h);
  const double s = f * ps;
  double pc = fma(z, -(h2 * h2 * h2) / 720, (h2 * h2) / 24);
  pc = fma(pc, z, -h2 / 2);
  const double c = fma(z, pc, 1.0);
  const double2 cst = lut64[kLnTab + lut_idx(i & 255u)];
  sn = fma(cst.y, c, cst.x * s);
  cs = fma(cst.x, c, -(cst.y * s));
}

// sin / cos of 2 pi r for a double phase r in revolutions (|r| < 2^20), full precision:
// n = rint(256 r), f = r - n / 256 exactly (Sterbenz), phi = 2 pi f in [-pi/256, pi/256];
// the series and the table of sincos_lut (LoS / two-path channel phases).  <= ~1.5 ulp.
__device__ __forceinline__ void sincos_rev_lut(double r, double& sn, double& cs) {
  const double n = __builtin_rint(256.0 * r);
  const double phi = (r - n * 0.00390625) * 6.28318530717958647693;
  const double z = phi * phi;
  double ps = fma(z, -1.0 / 5040, 1.0 / 120);
  ps = fma(ps, z, -1.0 / 6);
  const double s = fma(phi * z, ps, phi);
  double pc = fma(z, -1.0 / 720, 1.0 / 24);
  pc = fma(pc, z, -0.5);
  const double c = fma(z, pc, 1.0);
  const double2 cst = lut64[kLnTab + lut_idx((uint32_t)((int)n & 255))];
  sn = fma(cst.y, c, cst.x * s);
  cs = fma(cst.x, c, -(cst.y * s));
}

// ln u for u in (0, 1) (the Box-Muller radius argument): u = m 2^e with m in [0.5, 1) and
// e <= 0, so e ln 2 and ln m have the same sign and need no range fold; bucket i of m
// (the top 9 mantissa bits, width 2^-10) gives c_i ~ 1 / centre_i (12 bits; c = 1 for the
// top bucket: t = m - 1 exactly as u -> 1), t = m c_i - 1 with |t| < 2^-10, and
// log1p(t) to t^6 (truncation < 2^-60 relative).
// ESC: ln(x 2^ESC) -- the scale enters the exponent only (Box-Muller: x = w0 + 0.5, ESC = -32).
template <int ESC = 0>
__device__ __forceinline__ double ln_unit(double x) {
  // m and e by v_frexp_mant / v_frexp_exp (x normal, > 0): two instructions instead of the
  // bit surgery (shift, add; and, or and a register copy); the bucket from x's top mantissa bits
  const double m = __builtin_amdgcn_frexp_mant(x);
  const int e = __builtin_amdgcn_frexp_exp(x) + ESC;
  const uint32_t hi = (uint32_t)__double2hiint(x);
  const double2 cl = lut64[lut_idx((hi >> 11) & 511u)];
  const double t = fma(m, cl.x, -1.0);
  double q = -1.0 / 6;
  q = fma(q, t, 1.0 / 5);
  q = fma(q, t, -1.0 / 4);
  q = fma(q, t, 1.0 / 3);
  q = fma(q, t, -0.5);
  const double p = fma(t * t, q, t);
  constexpr double kLn2Hi = 6.93147180369123816490e-01;
  constexpr double kLn2Lo = 1.90821492927058770002e-10;
  const double de = (double)e;
  return fma(de, kLn2Hi, cl.y) + fma(de, kLn2Lo, p);
}
// sqrt of a positive normal double by the v_rsq_f64 seed (~2^-25) and one Newton step
// (~2^-49 relative).
__device__ __forceinline__ double sqrt_n1(double x) {
  const double r = __builtin_amdgcn_rsq(x);
  const double g = x * r, h = 0.5 * r;
  return fma(g, fma(-g, h, 0.5), g);
}
// 1/sqrt(x), x > 0 finite: seed and one Newton step (~2^-49 relative).
__device__ __forceinline__ double rsq_n1(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  return fma(y, fma(-0.5 * x * y, y, 0.5), y);
}

__device__ __forceinline__ float sin_rev(float r) { return __builtin_amdgcn_sinf(r); }
__device__ __forceinline__ float cos_rev(float r) { return __builtin_amdgcn_cosf(r); }

}  // namespace mimo
