// Workgroup ("team") FFT for the fused trial kernel — gfx950, fp32 or fp64 (Re).
//
// Replaces the reference's per-antenna torch CPU FFTs (modulation.py:270,
// utilities.py:329, corrector.py:93,98): ortho IFFT/FFT of one F-point OFDM symbol.
//
// Layout: the team has T threads (T = 64 * waves); thread t holds P = F/T complex
// points in registers in the CYCLIC distribution, element e at (thread e % T,
// register e / T).  A Stockham autosort radix-R stage reads, for butterfly
// j = t + T*i, the elements j + r*F/R = t + T*(i + r*P/R): all in the thread's own
// registers.  The last stage writes j + r*F/R as well, so input and output are both
// cyclic and a transform needs (stages - 1) exchanges through padded LDS buffers
// (one pad slot per 32 elements: conflict-free ds_write_b64 / ds_read_b64 for the
// stage patterns used here).  F = 2048 with P = 16 is radix 16 x 8 x 16 (plan below): two
// exchanges.
//
// Two alternating exchange buffers: one barrier per exchange (see stage()).
//
// Scaling is left to the caller (transforms are un-normalised).  DIR = -1 forward
// (e^{-j2pi nk/F}), +1 inverse.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "tuning.h"
#include "real.h"


namespace mimo {

// ---------------------------------------------------------------- compile-time trig
constexpr double kPi = 3.14159265358979323846264338327950288;

constexpr double ct_cos(double x) {
  while (x > kPi) x -= 2 * kPi;
  while (x < -kPi) x += 2 * kPi;
  double term = 1.0, sum = 1.0;
  for (int n = 1; n < 40; ++n) {
    term *= -x * x / ((2.0 * n - 1.0) * (2.0 * n));
    sum += term;
  }
  return sum;
}
constexpr double ct_sin(double x) { return ct_cos(x - kPi / 2); }

constexpr int ilog2(int n) { return n <= 1 ? 0 : 1 + ilog2(n >> 1); }

// ---------------------------------------------------------------- stage plan (host + device)
// F points, P per thread: NST Stockham stages; stage s has radix 2^bits(s) and
// NS = 2^bits_before(s).  Stage s >= 1 multiplies by twiddles exp(-j 2 pi jm r / (NS R)),
// jm < NS, 1 <= r < R, stored per stage as a [R][NS] block (lane-contiguous in jm) of
// one table; fft_tw_off(s) is the block's offset.
constexpr int fft_nst(int F, int P) { return (ilog2(F) + ilog2(P) - 1) / ilog2(P); }
// Radix plan: the last stage has radix P (one butterfly per thread, NS = T), the other
// bits are spread front-loaded over the earlier stages.  Every stage then has NS <= T, so
// the twiddles of a thread's butterflies i > 0 equal those of butterfly 0 (no compile-time
// rotations), e.g. F = 2048, P = 16: 16 x 8 x 16.  (The front-loaded 16 x 16 x 8 plan,
// whose last stage's second butterfly rotates, measured slower: git history.)
constexpr int fft_bits(int F, int P, int s) {
  if (fft_nst(F, P) > 1) {
    const int n = fft_nst(F, P) - 1, rest = ilog2(F) - ilog2(P);
    return s == n ? ilog2(P) : rest / n + (s < rest % n ? 1 : 0);
  }
  return ilog2(F);
}
constexpr int fft_bits_before(int F, int P, int s) { return s == 0 ? 0 : fft_bits_before(F, P, s - 1) + fft_bits(F, P, s - 1); }
constexpr int fft_tw_off(int F, int P, int s) {
  return s <= 1 ? 0 : fft_tw_off(F, P, s - 1) + (1 << (fft_bits_before(F, P, s - 1) + fft_bits(F, P, s - 1)));
}
constexpr int fft_tw_total(int F, int P) { return fft_tw_off(F, P, fft_nst(F, P)); }

template <class C>
__device__ __forceinline__ C cadd(C a, C b) {
  return mkc(a.x + b.x, a.y + b.y);
}
template <class C>
__device__ __forceinline__ C csub(C a, C b) {
  return mkc(a.x - b.x, a.y - b.y);
}
template <class C>
__device__ __forceinline__ C cmul(C a, C b) {
  return mkc(fmar(a.x, b.x, -a.y * b.y), fmar(a.x, b.y, a.y * b.x));
}
template <class C>
__device__ __forceinline__ C cmulc(C a, C b) {  // a * conj(b)
  return mkc(fmar(a.x, b.x, a.y * b.y), fmar(a.y, b.x, -a.x * b.y));
}
template <class C>
__device__ __forceinline__ C cmac(C acc, C a, C b) {  // acc + a * b, 4 FMAs
  return mkc(fmar(a.x, b.x, fmar(-a.y, b.y, acc.x)), fmar(a.x, b.y, fmar(a.y, b.x, acc.y)));
}
template <class C>
__device__ __forceinline__ C cscale(C a, real_of<C> s) {
  return mkc(a.x * s, a.y * s);
}

// x * exp(DIR * j * 2 pi * M / R) with the trivial angles resolved at compile time.
template <int M, int R, int DIR, class C>
__device__ __forceinline__ C ctw(C x) {
  using Re = real_of<C>;
  constexpr int m = ((M % R) + R) % R;
  if constexpr (m == 0) {
    return x;
  } else if constexpr (4 * m == R) {  // DIR * j
    return DIR > 0 ? mkc(-x.y, x.x) : mkc(x.y, -x.x);
  } else if constexpr (2 * m == R) {
    return mkc(-x.x, -x.y);
  } else if constexpr (4 * m == 3 * R) {  // -DIR * j
    return DIR > 0 ? mkc(x.y, -x.x) : mkc(-x.y, x.x);
  } else {
    constexpr Re c = (Re)ct_cos(2.0 * kPi * m / R);
    constexpr Re s = (Re)(DIR * ct_sin(2.0 * kPi * m / R));
    return mkc(fmar(x.x, c, -x.y * s), fmar(x.x, s, x.y * c));
  }
}

// x e^{DIR j 2pi K / 8} = c u for odd K, c = 1/sqrt(2): u (two adds) is returned and the
// caller folds c into the next additions as FMAs.
template <int K, int DIR, class C>
__device__ __forceinline__ C w8u(C x) {
  static_assert(K == 1 || K == 3, "odd multiples of pi/4");
  if constexpr (K == 1) return DIR < 0 ? mkc(x.x + x.y, x.y - x.x) : mkc(x.x - x.y, x.x + x.y);
  else return DIR < 0 ? mkc(x.y - x.x, -x.x - x.y) : mkc(-x.x - x.y, x.x - x.y);
}
template <class C>
__device__ __forceinline__ C cfma(real_of<C> c, C u, C a) {  // a + c u
  return mkc(fmar(c, u.x, a.x), fmar(c, u.y, a.y));
}
constexpr double kRsqrt2 = 0.70710678118654752440084436210484903928;

// a + b / a - b where inputs known to be zero at compile time (ZA, ZB) are skipped:
// pruning the IFFT's structurally-zero out-of-band inputs.
template <bool ZA, bool ZB, class C>
__device__ __forceinline__ C zadd(C a, C b) {
  if constexpr (ZA && ZB) return czero<real_of<C>>();
  else if constexpr (ZA) return b;
  else if constexpr (ZB) return a;
  else return cadd(a, b);
}
template <bool ZA, bool ZB, class C>
__device__ __forceinline__ C zsub(C a, C b) {
  if constexpr (ZA && ZB) return czero<real_of<C>>();
  else if constexpr (ZA) return mkc(-b.x, -b.y);
  else if constexpr (ZB) return a;
  else return csub(a, b);
}

// In-register DFT of size R (natural order in and out), four-step R = R1 x R2.
// ZM: bit n set = input n is zero for every thread (compile-time pruning).
template <int R, int DIR, uint32_t ZM = 0>
struct Dft {
  static constexpr bool z(int n) { return ((ZM >> n) & 1u) != 0; }
  static constexpr uint32_t sub_mask(int n1, int r1, int r2) {
    uint32_t m = 0;
    for (int n2 = 0; n2 < r2; ++n2) m |= ((ZM >> (n1 + r1 * n2)) & 1u) << n2;
    return m;
  }
  template <int N1, int R1, int R2, class C>
  static __device__ __forceinline__ void first_level(C (&sub)[R1][R2], const C* v) {
    if constexpr (N1 < R1) {
#pragma unroll
      for (int n2 = 0; n2 < R2; ++n2) sub[N1][n2] = v[N1 + R1 * n2];
      Dft<R2, DIR, sub_mask(N1, R1, R2)>::run(sub[N1]);
      first_level<N1 + 1, R1, R2>(sub, v);
    }
  }

  template <class C>
  static __device__ __forceinline__ void run(C* v) {
    if constexpr (R == 1) {
      return;
    } else if constexpr (R == 2) {
      const C a = v[0], b = v[1];
      v[0] = zadd<z(0), z(1)>(a, b);
      v[1] = zsub<z(0), z(1)>(a, b);
    } else if constexpr (R == 4) {
      constexpr bool z02 = z(0) && z(2), z13 = z(1) && z(3);
      const C t0 = zadd<z(0), z(2)>(v[0], v[2]), t1 = zsub<z(0), z(2)>(v[0], v[2]);
      const C t2 = zadd<z(1), z(3)>(v[1], v[3]);
      const C t3 = z13 ? czero<real_of<C>>() : ctw<1, 4, DIR>(zsub<z(1), z(3)>(v[1], v[3]));
      v[0] = zadd<z02, z13>(t0, t2);
      v[2] = zsub<z02, z13>(t0, t2);
      v[1] = zadd<z02, z13>(t1, t3);
      v[3] = zsub<z02, z13>(t1, t3);
    } else if constexpr (R == 8) {
      // 2 x 4: two DFT-4s, then the DFT-2s with W8^k2 on the odd half.  The odd-multiple-
      // of-pi/4 rotations W8^1, W8^3 are c (+-x.x +- x.y, +-x.x +- x.y), c = 1/sqrt(2):
      // two adds, and c goes into the DFT-2 as an FMA (6 ops instead of 4 + 4).
      C sub[2][4];
      first_level<0, 2, 4>(sub, v);
      using Re = real_of<C>;
      constexpr Re c = (Re)kRsqrt2;
#pragma unroll
      for (int k2 = 0; k2 < 4; ++k2) {
        const C a = sub[0][k2], x = sub[1][k2];
        if (k2 == 0 || k2 == 2) {
          const C b = k2 == 0 ? x : ctw<2, 8, DIR>(x);
          v[k2] = cadd(a, b);
          v[k2 + 4] = csub(a, b);
        } else {
          const C u = k2 == 1 ? w8u<1, DIR>(x) : w8u<3, DIR>(x);  // x e^{DIR j 2pi k2 / 8} = c u
          v[k2] = cfma(c, u, a);
          v[k2 + 4] = cfma(-c, u, a);
        }
      }
    } else if constexpr (R == 16) {
      // 4 x 4 four-step.  Of the inter-step twiddles W16^(n1 k2), W16^2 and W16^6 are
      // W8-type rotations c u: u costs two adds and c goes into the column DFT-4's
      // additions as FMAs (8 ops fewer per DFT-16 than four generic rotations).
      C sub[4][4];
      first_level<0, 4, 4>(sub, v);
      using Re = real_of<C>;
      constexpr Re c = (Re)kRsqrt2;
      {  // column 0: no twiddles
        C col[4] = {sub[0][0], sub[1][0], sub[2][0], sub[3][0]};
        Dft<4, DIR>::run(col);
#pragma unroll
        for (int k1 = 0; k1 < 4; ++k1) v[4 * k1] = col[k1];
      }
      // columns 1 and 3: n1 = 2 carries W16^2 / W16^6 (= W8^1 / W8^3)
      auto odd_col = [&](auto k2c) __attribute__((always_inline)) {
        constexpr int K2 = decltype(k2c)::value;
        const C x0 = sub[0][K2];
        const C u2 = w8u<K2 == 1 ? 1 : 3, DIR>(sub[2][K2]);
        const C x1 = ctw<K2, 16, DIR>(sub[1][K2]), x3 = ctw<3 * K2, 16, DIR>(sub[3][K2]);
        const C t0 = cfma(c, u2, x0), t1 = cfma(-c, u2, x0);
        const C t2 = cadd(x1, x3), t3 = ctw<1, 4, DIR>(csub(x1, x3));
        v[K2] = cadd(t0, t2);
        v[K2 + 8] = csub(t0, t2);
        v[K2 + 4] = cadd(t1, t3);
        v[K2 + 12] = csub(t1, t3);
      };
      odd_col(std::integral_constant<int, 1>{});
      odd_col(std::integral_constant<int, 3>{});
      {  // column 2: W16^2 (n1 = 1), W16^4 = DIR j (n1 = 2), W16^6 (n1 = 3)
        const C x0 = sub[0][2], x2 = ctw<4, 16, DIR>(sub[2][2]);
        const C u1 = w8u<1, DIR>(sub[1][2]), u3 = w8u<3, DIR>(sub[3][2]);
        const C t0 = cadd(x0, x2), t1 = csub(x0, x2);
        const C sp = cadd(u1, u3), sm = ctw<1, 4, DIR>(csub(u1, u3));  // t2 = c sp, t3 = c sm
        v[2] = cfma(c, sp, t0);
        v[10] = cfma(-c, sp, t0);
        v[6] = cfma(c, sm, t1);
        v[14] = cfma(-c, sm, t1);
      }
    } else {
      constexpr int R1 = (R >= 16) ? 4 : 2;
      constexpr int R2 = R / R1;
      C sub[R1][R2];
      first_level<0, R1, R2>(sub, v);
      Twid<R1, R2, 1, 0>::apply(sub);
#pragma unroll
      for (int k2 = 0; k2 < R2; ++k2) {
        C col[R1];
#pragma unroll
        for (int n1 = 0; n1 < R1; ++n1) col[n1] = sub[n1][k2];
        Dft<R1, DIR>::run(col);
#pragma unroll
        for (int k1 = 0; k1 < R1; ++k1) v[k2 + R2 * k1] = col[k1];
      }
    }
  }

  // sub[n1][k2] *= W_R^(n1 k2), unrolled with compile-time indices.
  template <int R1, int R2, int N1, int K2>
  struct Twid {
    template <typename A>
    static __device__ __forceinline__ void apply(A& sub) {
      if constexpr (N1 < R1) {
        if constexpr (K2 < R2) {
          sub[N1][K2] = ctw<N1 * K2, R, DIR>(sub[N1][K2]);
          Twid<R1, R2, N1, K2 + 1>::apply(sub);
        } else {
          Twid<R1, R2, N1 + 1, 0>::apply(sub);
        }
      }
    }
  };
};

// ---------------------------------------------------------------- twiddles absorbed into FMAs
// A twiddle z = c + j s stored as (c, t = s / c) ("cot-tan" form): z b = c (b + j t b), so a
// radix-2 butterfly a +- z b is u = (b.x - t b.y, b.y + t b.x) and a +- c u -- 6 FMAs instead
// of a complex multiply (2 mul + 2 fma) and 4 additions.  The inverse uses conj(z): t -> -t.
// ROT: the twiddle times rho = DIR j (W_4 of the transform's direction) -- operands swapped,
// still 6 FMAs.  Exact in the limit c -> 0 as long as c != 0 (the host tables hold
// cos(pi/2) = 6.1e-17, never 0): c t rounds to s, and the dropped b term is c b ~ 1e-16 b.
template <int DIR, bool ROT, class C, typename Re = real_of<C>>
__device__ __forceinline__ void bfly_ct(C a, C b, C ct, C& o0, C& o1) {
  const Re c = ct.x, tt = DIR < 0 ? ct.y : -ct.y;
  const Re ux = fmar(-tt, b.y, b.x), uy = fmar(tt, b.x, b.y);
  if constexpr (!ROT) {
    o0 = mkc(fmar(c, ux, a.x), fmar(c, uy, a.y));
    o1 = mkc(fmar(-c, ux, a.x), fmar(-c, uy, a.y));
  } else {
    const Re cd = DIR < 0 ? -c : c;  // rho c u = cd (-u.y, u.x)
    o0 = mkc(fmar(-cd, uy, a.x), fmar(cd, ux, a.y));
    o1 = mkc(fmar(cd, uy, a.x), fmar(-cd, ux, a.y));
  }
}
// y[k] = sum_r W8^(r k) z^r v[r] (natural order in and out) as three radix-2 DIT levels with
// every twiddle absorbed (12 butterflies = 72 FMAs, against 7 complex multiplies + the
// 52-op DFT-8 = 80): level 1 pairs (r, r + 4) with z^4, level 2 (r0, r0 + 2) with
// W4^k0 z^2, level 3 (0, 1) with W8^m z.  zc: (c, t) of z^4, z^2, z and W8 z (forward W8 =
// e^{-j pi / 4}; the inverse conjugates all of them).
template <int DIR, class C>
__device__ __forceinline__ void dft8_ct(C (&v)[8], const C (&zc)[4]) {
  C a0[4], a1[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) bfly_ct<DIR, false>(v[r], v[r + 4], zc[0], a0[r], a1[r]);
  C b[2][4];
#pragma unroll
  for (int r0 = 0; r0 < 2; ++r0) {
    bfly_ct<DIR, false>(a0[r0], a0[r0 + 2], zc[1], b[r0][0], b[r0][2]);
    bfly_ct<DIR, true>(a1[r0], a1[r0 + 2], zc[1], b[r0][1], b[r0][3]);
  }
  bfly_ct<DIR, false>(b[0][0], b[1][0], zc[2], v[0], v[4]);
  bfly_ct<DIR, true>(b[0][2], b[1][2], zc[2], v[2], v[6]);
  bfly_ct<DIR, false>(b[0][1], b[1][1], zc[3], v[1], v[5]);
  bfly_ct<DIR, true>(b[0][3], b[1][3], zc[3], v[3], v[7]);
}
// The same for R = 16 (four levels, 32 butterflies = 192 FMAs, against 15 complex
// multiplies, the products forming 11 of the 15 twiddles and the ~152-op DFT-16): level 1
// (r, r + 8) with z^8, level 2 (r, r + 4) with W4^k0 z^4, level 3 (r0, r0 + 2) with W8^m z^2,
// level 4 (0, 1) with W16^m z.  zc: (c, t) of z^8, z^4, z^2, W8 z^2, z, W16 z, W8 z, W16^3 z.
// (Forming the rotated rows from z^2 and z in registers instead -- 4 table rows, +2 ops on
// 10 butterflies -- measured +1 to +4 %, profiles/r05/ab/ab_*_r05e.json: not taken.)
template <int DIR, class C>
__device__ __forceinline__ void dft16_ct(C (&v)[16], const C (&zc)[8]) {
  C a[2][8];
#pragma unroll
  for (int r = 0; r < 8; ++r) bfly_ct<DIR, false>(v[r], v[r + 8], zc[0], a[0][r], a[1][r]);
  C b[4][4];  // b[r][m], m = k mod 4
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    bfly_ct<DIR, false>(a[0][r], a[0][r + 4], zc[1], b[r][0], b[r][2]);
    bfly_ct<DIR, true>(a[1][r], a[1][r + 4], zc[1], b[r][1], b[r][3]);
  }
  C c[2][8];  // c[r0][m], m = k mod 8
#pragma unroll
  for (int r0 = 0; r0 < 2; ++r0) {
    bfly_ct<DIR, false>(b[r0][0], b[r0 + 2][0], zc[2], c[r0][0], c[r0][4]);
    bfly_ct<DIR, true>(b[r0][2], b[r0 + 2][2], zc[2], c[r0][2], c[r0][6]);
    bfly_ct<DIR, false>(b[r0][1], b[r0 + 2][1], zc[3], c[r0][1], c[r0][5]);
    bfly_ct<DIR, true>(b[r0][3], b[r0 + 2][3], zc[3], c[r0][3], c[r0][7]);
  }
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    bfly_ct<DIR, false>(c[0][m], c[1][m], zc[4 + m], v[m], v[m + 8]);
    bfly_ct<DIR, true>(c[0][m + 4], c[1][m + 4], zc[4 + m], v[m + 4], v[m + 12]);
  }
}
// Host / device: the cot-tan rows of a radix-R stage (R = 8: 4 rows, 16: 8 rows), lane jm,
// z = exp(-j 2 pi jm / (R NS)), as angles in revolutions (ct_rows, ct_rev).
__host__ __device__ constexpr int ct_rows(int R) { return R == 8 ? 4 : 8; }
// entries of a transform's cot-tan region: stage s >= 1, [ct_rows][NS_s] (c, tan) each
constexpr int fft_ct_n(int F, int P) {
  int n = 0;
  for (int s = 1; s < fft_nst(F, P); ++s) n += ct_rows(1 << fft_bits(F, P, s)) * (1 << fft_bits_before(F, P, s));
  return n;
}
__host__ __device__ constexpr double ct_rev(int R, int ns, int jm, int q) {
  const double th = -(double)jm / ((double)R * ns);
  if (R == 8) return q == 0 ? 4 * th : q == 1 ? 2 * th : q == 2 ? th : th - 0.125;
  switch (q) {
    case 0: return 8 * th;
    case 1: return 4 * th;
    case 2: return 2 * th;
    case 3: return 2 * th - 0.125;
    case 4: return th;
    case 5: return th - 0.0625;
    case 6: return th - 0.125;
    default: return th - 0.1875;
  }
}

// Exchange synchronisation: the whole team (s_barrier) or, for a one-wave transform
// (WAVE, wave_fft.h), the wave alone.  A wave's LDS instructions execute in issue order,
// so its own exchanges need only a compiler-level fence, no hardware barrier.
template <bool WAVE>
__device__ __forceinline__ void xchg_sync() {
  if constexpr (WAVE) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
}

// ---------------------------------------------------------------- team FFT
// LTW1: stage 1's twiddle block comes from an LDS copy (run()'s tw1 argument; the wave-split
// FFT's one-wave sub-transforms, whose stage-1 block is small: 64 entries at F 2048) -- all
// R - 1 twiddles read, none formed as products (fp64: 16 VALU ops per stage saved).
template <int F, int T, int NBUF = 2, typename Re = float, bool WAVE = false, bool LTW1 = false, bool LTW2_ON = false,
          bool CT_ON = false>
struct TeamFft {
  using C = cx<Re>;
  static constexpr int P = F / T;
  static constexpr int LOG_F = ilog2(F);
  static constexpr int LOG_P = ilog2(P);
  static constexpr int NST = fft_nst(F, P);
  // Padding of exchange S: one slot per 2^PSH elements.  Exchange 0 (stage 0 writes
  // 16t + r) uses 1/16: it halves that exchange's modelled bank
  // conflicts (tools/lds_conflicts.py); later exchanges use 1/32.
  // fp64 elements are 16 B (ds_write_b128: 8-lane groups over 32 banks), where stage 0's
  // stride-R writes need one pad slot per 8 elements: the modelled extra LDS cycles of
  // exchange 0 drop 3x (tools/lds_conflicts.py; the model reproduces SQ_LDS_BANK_CONFLICT
  // of the 1/16 layout exactly, profiles/r02/pmc_f64_r1).  F = 8192 keeps 1/16: its 16 KiB
  // more would not fit the 160 KiB LDS next to the fp64 tables and the CSI scratch.
  // Exchanges >= 1: one pad slot per 32 elements; fp64 from F 4096 one per 128 (modelled
  // conflict-free as well, tests/test_lds_layout.py: 3 KiB of LDS back at F 8192).
  static constexpr int PADN = (sizeof(Re) == 8 && F >= 4096) ? 7 : 5;
  // (fp64 F 4096 on 256 threads: 1/32, so that two teams fit a CU -- 80,256 B each)
  static constexpr int PAD0 = (sizeof(Re) == 8 && F < 8192) ? (F == 4096 && T == 256 ? 5 : 3) : 4;
  static constexpr int psh(int S) { return S == 0 ? PAD0 : PADN; }
  // Exchange 0 transposed (XP0): stage 0 (NS = 1) writes element e = R0 j + r, which the
  // linear layouts above put R0 elements apart in consecutive lanes (an R0-element stride
  // is a multiple of the 8 x 16-B bank groups of ds_write_b128: 8-way conflicts unpadded,
  // 2-way at 1/16, 1/8 of the buffer to remove them).  Stored as [R0][F / R0 + XD0]
  // (address (e % R0) XS0 + e / R0) the writes of one r are consecutive in the lanes and
  // stage 1's reads (e = t + T m) land on 16 distinct 16-B bank groups per read group:
  // conflict-free for XD0 = 32 / R0 (R0 = 4: 4 in fp64, 8 in fp32) in both precisions
  // (tools/lds_conflicts.py --xpose, tests/test_lds_layout.py), for R0 XD0 <= 32 extra
  // elements instead of F / 16.
  static constexpr int R0 = NST > 1 ? 1 << fft_bits(F, P, 0) : 1;
  static constexpr bool XP0 = NST > 1 && R0 >= 4 && R0 <= 16 && T % R0 == 0;
  static constexpr int XD0 = !XP0 ? 0 : R0 == 4 ? (sizeof(Re) == 8 ? 4 : 8) : 32 / R0;
  static constexpr int XS0 = F / R0 + XD0;  // row stride of the transposed exchange 0
  static constexpr int lin_elems(int sh) { return F + F / (1 << sh); }
  static constexpr int LDS_ELEMS = XP0 ? (R0 * XS0 > lin_elems(PADN) ? R0 * XS0 : lin_elems(PADN))
                                       : lin_elems(PAD0 < PADN ? PAD0 : PADN);
  static_assert((1 << LOG_F) == F && (1 << LOG_P) == P && P >= 2, "power-of-two sizes");
  static_assert(!WAVE || T == 64, "wave-local transforms are one wave");

  static constexpr int bits(int s) { return fft_bits(F, P, s); }
  static constexpr int bits_before(int s) { return fft_bits_before(F, P, s); }
  // entries of stage 1's [R][NS] twiddle block (offset 0 of the table)
  static constexpr int TW1_N = NST > 1 ? (1 << fft_bits(F, P, 1)) * (1 << fft_bits_before(F, P, 1)) : 1;
  // With LTW2_ON a radix-8 stage 2 also reads its non-power-of-two twiddles r = 3, 5, 6 from
  // the LDS copy (rows [3][NS] after stage 1's block; r = 7 stays the product w4 w3): 3 of
  // its 4 twiddle products per transform gone.  (All four rows would not fit next to the
  // fp64 F 2048 team's 3-teams-per-CU LDS line.)
  static constexpr bool LTW2 = LTW1 && LTW2_ON && NST >= 3 && fft_bits(F, P, 2) == 3;
  static constexpr int NS2 = NST >= 3 ? 1 << fft_bits_before(F, P, 2) : 1;
  // CT (fp64): every twiddled stage (radix 8 or 16) runs dft8_ct / dft16_ct on cot-tan
  // constants, [ct_rows][NS] per stage at ct_off(s) of the cot-tan region: in the LDS copy
  // for the wave-local sub-transforms (which then replace stage 1's block and stage 2's
  // rows; both stages must fit), else read from global memory after the stage twiddle table
  // (fft_tw_total).  A thread's butterflies share one twiddle set (NS <= T, tw_shift's OFF = 0).
  static constexpr bool ct_ok() {
    for (int s = 1; s < NST; ++s)
      if (fft_bits(F, P, s) != 3 && fft_bits(F, P, s) != 4) return false;
    return NST >= 2;
  }
  static constexpr bool CT = CT_ON && sizeof(Re) == 8 && ct_ok() && (!WAVE || (LTW1 && LTW2 && NST == 3));
  static constexpr int ct_off(int s) {
    return s <= 1 ? 0
                  : ct_off(s - 1) + ct_rows(1 << fft_bits(F, P, s - 1)) * (1 << fft_bits_before(F, P, s - 1));
  }
  static constexpr int CT_N = CT ? ct_off(NST) : 0;  // cot-tan entries
  // (Team FFT variants measured and not taken, profiles/r05/ab/ab_*_r05e.json: the radix-16
  // stages only, stage 1's constants from an LDS copy.)
  static constexpr bool ct_stage(int s) { return CT && s >= 1; }
  // CT_PF (A/B knob MIMO_CT_PF): the global-memory cot-tan constants of stage s + 1 loaded
  // before stage s's exchange (their L2 latency under the barrier and the LDS round trip)
  // instead of at the top of stage s + 1.  Off: paper +1.6 %, paper CNC 0-8 +1.7 %, config-5
  // array +5.3 % with it (the constants held across the exchange; profiles/r06/k4096/,
  // k8192/ab_5su_ctpf.json).
  static constexpr bool CT_PF = MIMO_CT_PF != 0 && CT && !WAVE;
  template <int S>
  static __device__ __forceinline__ void load_ct(C (&w)[8], const C* __restrict__ tw, int t) {
    constexpr int NS = 1 << bits_before(S);
    constexpr int Q = ct_rows(1 << bits(S));
    const C* cts = tw + fft_tw_total(F, P) + ct_off(S);
    const int jm0 = t & (NS - 1);
#pragma unroll
    for (int q = 0; q < Q; ++q) w[q] = gload(cts + q * NS, jm0);
  }
  static constexpr int TWL_N = CT && WAVE ? CT_N : TW1_N + (LTW2 ? 3 * NS2 : 0);  // LDS copy
  // source index in the twiddle table of LDS-copy entry i < TWL_N (CT: relative to the
  // cot-tan region, which the caller's table places)
  static __host__ __device__ constexpr int twl_src(int i) {
    if ((CT && WAVE) || i < TW1_N) return i;
    const int j = i - TW1_N, row = j / NS2, r = row == 0 ? 3 : row == 1 ? 5 : 6;
    return fft_tw_off(F, P, 2) + r * NS2 + j % NS2;
  }
  template <int S>
  static __host__ __device__ constexpr int pad(int e) { return e + (e >> psh(S)); }
  // Global-address-space load (the laundered table pointer would otherwise be generic
  // and compile to flat loads, which also count against lgkmcnt with the LDS traffic).
  static __device__ __forceinline__ C gload(const C* p, int i) {
    typedef Re v2f __attribute__((ext_vector_type(2)));
    const v2f v = ((const __attribute__((address_space(1))) v2f*)p)[i];
    return mkc(v.x, v.y);
  }

  // Twiddles of stage S for butterflies i > 0: jm_i = jm_0 + OFF_i with OFF_i = (T i) mod NS
  // (T and NS are powers of two, t < T), so w_i[r] = w_0[r] exp(-j 2 pi OFF_i r / (NS R)):
  // a compile-time rotation instead of a load.
  template <int N, int OFF, int R, int r = 1>
  static __device__ __forceinline__ void tw_shift(C (&w)[R], const C (&w0)[R]) {
    if constexpr (r < R) {
      w[r] = ctw<OFF * r, N, -1>(w0[r]);
      tw_shift<N, OFF, R, r + 1>(w, w0);
    }
  }

  // One radix-R butterfly (index i of the thread's B) of stage S.
  // Zero mask of butterfly I's inputs v[r] = d[I + r B] from the register mask ZM.
  static constexpr uint32_t bfly_mask(uint32_t zm, int i, int b, int r) {
    uint32_t m = 0;
    for (int k = 0; k < r; ++k) m |= ((zm >> (i + k * b)) & 1u) << k;
    return m;
  }

  template <int S, int DIR, int I, uint32_t ZM>
  static __device__ __forceinline__ void butterfly(C (&d)[P], C* buf, const C (&w0)[1 << bits(S)],
                                                   int t, bool no_xchg) {
    constexpr int R = 1 << bits(S);
    constexpr int NS = 1 << bits_before(S);
    constexpr int B = P / R;
    constexpr bool LAST = (S == NST - 1);
    C v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = d[I + r * B];
    const int j = t + T * I;
    const int jm = j & (NS - 1);
    if constexpr (ct_stage(S)) {
      if constexpr (R == 8) {
        const C zc[4] = {w0[0], w0[1], w0[2], w0[3]};
        dft8_ct<DIR>(v, zc);
      } else {
        const C zc[8] = {w0[0], w0[1], w0[2], w0[3], w0[4], w0[5], w0[6], w0[7]};
        dft16_ct<DIR>(v, zc);
      }
    } else if constexpr (NS > 1) {
      constexpr int OFF = (T * I) & (NS - 1);
      C w[R];
      if constexpr (OFF == 0) {
#pragma unroll
        for (int r = 1; r < R; ++r) w[r] = w0[r];
      } else {
        tw_shift<NS * R, OFF, R>(w, w0);
      }
#pragma unroll
      for (int r = 1; r < R; ++r) v[r] = DIR < 0 ? cmul(v[r], w[r]) : cmulc(v[r], w[r]);
    }
    if constexpr (!ct_stage(S)) Dft<R, DIR, (S == 0 ? bfly_mask(ZM, I, B, R) : 0u)>::run(v);
    if constexpr (LAST) {
#pragma unroll
      for (int r = 0; r < R; ++r) d[I + r * B] = v[r];
    } else if (no_xchg) {  // ablation: data stay in registers (wrong result, no LDS / barriers)
#pragma unroll
      for (int r = 0; r < R; ++r) d[I + r * B] = v[r];
    } else {
      // One buffer: everyone must have read the previous exchange before it is
      // overwritten.  The barrier sits after this stage's twiddle loads and DFT, so
      // their latency overlaps the previous exchange's reads.
      if constexpr (NBUF == 1 && I == 0) xchg_sync<WAVE>();
      if constexpr (S == 0 && XP0) {
        // transposed exchange 0: element R j + r at r XS0 + j
        C* wb = buf + j;
#pragma unroll
        for (int r = 0; r < R; ++r) wb[r * XS0] = v[r];
      } else {
        // pad(base + r NS) == pad(base) + pad(r NS) for power-of-two NS, R, T (the
        // padding never splits a write group): one address per i, immediate offsets.
        C* wb = buf + pad<S>((j / NS) * NS * R + jm);
#pragma unroll
        for (int r = 0; r < R; ++r) wb[pad<S>(r * NS)] = v[r];
      }
    }
  }

  template <int S, int DIR, uint32_t ZM, int I = 0>
  static __device__ __forceinline__ void butterflies(C (&d)[P], C* buf, const C (&w0)[1 << bits(S)],
                                                     int t, bool no_xchg) {
    if constexpr (I < P / (1 << bits(S))) {
      butterfly<S, DIR, I, ZM>(d, buf, w0, t, no_xchg);
      butterflies<S, DIR, ZM, I + 1>(d, buf, w0, t, no_xchg);
    }
  }

  // Exchange buffers alternate (stage S of a transform started at parity PAR uses buffer
  // (S + PAR) & 1), so a write never targets the buffer other threads may still be
  // reading: before a thread writes buffer X for exchange k+2 it has passed the barrier
  // of exchange k+1, which every thread reaches only after reading X for exchange k.
  // One barrier per exchange.  Callers keep the number of exchanges between two
  // transforms' parities consistent (an antenna = IFFT + FFT = an even count).
  //
  // Twiddles: the [R][NS] block of stage S gives w(jm, r) = exp(-j 2 pi jm r / (NS R)).
  // Only r = 1, 2, 4, ... are loaded (uniform base per r in SGPRs + the lane's jm as the
  // VGPR offset); the other r are products w(jm, a) w(jm, b), a + b = r (at most
  // log2 R - 1 roundings).  Loads, not multiplies, were the twiddles' cost: dropping the
  // loads saved 17 % of the kernel, dropping the multiplies 8 % (profiles/r01).
  // Base twiddles w(jm0, 2^b) of every stage >= 1, loaded together at the start of a
  // transform (PREFETCH): their L2 latency then overlaps stage 0 and the first
  // exchange instead of stalling each stage's first twiddle multiply.
  static constexpr int kMaxB = 5;
  // Measured -1.1 % (F 2048), -1.5 % (F 4096), +0.9 % (F 8192: more stages held live);
  // fp64: -2.4 % at F = 2048 (with the channel pipeline off), +1.5 % at F = 4096
  // (profiles/r02/ab/ab64_*.json).
  // fp64 F 8192 (16 points per thread): -2.2 % (profiles/r03/ab8k/ab_diet_prefetch.json).
  static constexpr bool PREFETCH = (F <= 4096 && (sizeof(Re) == 4 || F <= 2048)) || (sizeof(Re) == 8 && F >= 8192);
  // Base holds w(2^k) for k < kMaxB; a stage reads k < bits(S) <= LOG_P.
  static_assert(!PREFETCH || LOG_P <= kMaxB, "Base too small for the plan's largest radix");
  struct Base {
    C v[NST][kMaxB];
  };
  template <int S>
  static __device__ __forceinline__ void load_base(Base& b, const C* __restrict__ tw, int t) {
    if constexpr (S < NST) {
      constexpr int R = 1 << bits(S);
      constexpr int NS = 1 << bits_before(S);
      if constexpr (NS > 1 && !(LTW1 && S == 1) && !ct_stage(S)) {
        constexpr int TW_OFF = fft_tw_off(F, P, S);
        const int jm0 = t & (NS - 1);
#pragma unroll
        for (int k = 0; k < bits(S) && k < kMaxB; ++k)
          b.v[S][k] = gload(tw + TW_OFF + (1 << k) * NS, jm0);
        (void)R;
      }
      load_base<S + 1>(b, tw, t);
    }
  }

  template <int S, int DIR, int PAR, uint32_t ZM, typename Fill>
  static __device__ __forceinline__ void stage(C (&d)[P], C* lds, const C* __restrict__ tw, int t,
                                               bool no_xchg, const Base& base, const Fill& fill,
                                               const C* tw1, C (&wct)[8]) {
    constexpr int R = 1 << bits(S);
    constexpr int NS = 1 << bits_before(S);
    constexpr int B = P / R;
    constexpr bool LAST = (S == NST - 1);
    static_assert(B >= 1 && B * R == P, "radix must divide points per thread");
    C* buf = lds + (NBUF == 2 ? ((S + PAR) & 1) * LDS_ELEMS : 0);
    C w0[R];
    if constexpr (ct_stage(S)) {
      // cot-tan constants in w0[0 .. ct_rows) (butterfly() runs dft8_ct / dft16_ct)
      static_assert(((T * (B - 1)) & (NS - 1)) == 0, "cot-tan stages: one twiddle set per thread");
      constexpr int Q = ct_rows(R);
      if constexpr (CT_PF) {
#pragma unroll
        for (int q = 0; q < Q; ++q) w0[q] = wct[q];  // loaded before the previous exchange
      } else if constexpr (WAVE) {
        const C* cts = tw1 + ct_off(S) + (t & (NS - 1));
#pragma unroll
        for (int q = 0; q < Q; ++q) w0[q] = cts[q * NS];
      } else {
        const C* cts = tw + fft_tw_total(F, P) + ct_off(S);
        const int jm0 = t & (NS - 1);
#pragma unroll
        for (int q = 0; q < Q; ++q) w0[q] = gload(cts + q * NS, jm0);
      }
    } else if constexpr (NS > 1 && LTW1 && S == 1) {
      const C* tws = tw1 + (t & (NS - 1));
#pragma unroll
      for (int r = 1; r < R; ++r) w0[r] = tws[r * NS];
    } else if constexpr (NS > 1 && PREFETCH) {
#pragma unroll
      for (int r = 1; r < R; ++r) {
        if ((r & (r - 1)) == 0) {
          w0[r] = base.v[S][ilog2(r)];
        } else if (LTW2 && S == 2 && r != 7) {
          w0[r] = tw1[TW1_N + (r == 3 ? 0 : r == 5 ? 1 : 2) * NS + (t & (NS - 1))];
        } else {
          int hb = r;
          while (hb & (hb - 1)) hb &= hb - 1;
          w0[r] = cmul(w0[hb], w0[r - hb]);
        }
      }
    } else if constexpr (NS > 1) {
      constexpr int TW_OFF = fft_tw_off(F, P, S);  // forced compile-time (a runtime call otherwise)
      const C* tws = tw + TW_OFF;
      const int jm0 = t & (NS - 1);
#pragma unroll
      for (int r = 1; r < R; ++r) {
        if ((r & (r - 1)) == 0) {
          w0[r] = gload(tws + r * NS, jm0);
        } else {
          int hb = r;
          while (hb & (hb - 1)) hb &= hb - 1;  // highest power of two below r (unrolled: constant)
          w0[r] = cmul(w0[hb], w0[r - hb]);
        }
      }
    }
    butterflies<S, DIR, ZM>(d, buf, w0, t, no_xchg);
    if constexpr (!LAST) {
      if constexpr (CT_PF && ct_stage(S + 1)) load_ct<S + 1>(wct, tw, t);
      if (!no_xchg) {
        xchg_sync<WAVE>();
        if constexpr (S == 0 && XP0) {
          // element t + T m at (t % R0) XS0 + t / R0 + (T / R0) m
          const C* rb = buf + (t % R0) * XS0 + t / R0;
#pragma unroll
          for (int m = 0; m < P; ++m) d[m] = rb[(T / R0) * m];
        } else {
          const C* rb = buf + pad<S>(t);
#pragma unroll
          for (int m = 0; m < P; ++m) d[m] = rb[pad<S>(T * m)];
        }
      }
      // Independent caller work placed between this exchange's reads and their first use
      // (same basic block: the scheduler interleaves it with the LDS latency).
      fill(S);
    }
  }

  template <int S, int DIR, int PAR, uint32_t ZM, typename Fill>
  static __device__ __forceinline__ void stages(C (&d)[P], C* lds, const C* __restrict__ tw, int t,
                                                bool no_xchg, const Base& base, const Fill& fill, const C* tw1,
                                                C (&wct)[8]) {
    if constexpr (S < NST) {
      stage<S, DIR, PAR, ZM>(d, lds, tw, t, no_xchg, base, fill, tw1, wct);
      stages<S + 1, DIR, PAR, ZM>(d, lds, tw, t, no_xchg, base, fill, tw1, wct);
    }
  }

  static constexpr int XCHG = NST - 1;  // exchanges per transform
  // The frequency-domain vector is cyclic in the thread id itself (split_fft.h permutes it).
  static __device__ __forceinline__ int freq_thread(int t) { return t; }
  static constexpr int LDS_TOTAL = NBUF * LDS_ELEMS;  // exchange buffer(s)

  // Un-normalised transform of the team's cyclic-distributed vector.  Ends with the
  // last exchange's reads done by this thread only: callers that touch `lds` next must
  // barrier first (the next transform's first exchange does).
  //
  // The twiddles and LDS addresses depend only on the thread id, so inside the
  // caller's antenna loop LICM would hoist all of them (~60 VGPRs) out of the loop and
  // spill.  Laundering t and tw through empty asm makes them opaque per transform:
  // they are re-derived (cheap ALU + L1-hit loads) instead of held.
  //
  // ZM: registers d[m] (bit m) that are zero in every thread on entry (the IFFT's
  // out-of-band bins); stage 0 skips their additions.
  struct NoFill {
    __device__ __forceinline__ void operator()(int) const {}
  };
  template <int DIR, int PAR = 0, uint32_t ZM = 0, typename Fill = NoFill>
  static __device__ __forceinline__ void run(C (&d)[P], C* lds, const C* __restrict__ tw, int t,
                                             bool no_xchg = false, const Fill& fill = Fill{},
                                             const C* tw1 = nullptr) {
    const C* twl = tw;
    int tl = t;
    asm volatile("" : "+s"(twl));
    asm volatile("" : "+v"(tl));
    Base base;
    if constexpr (PREFETCH) load_base<1>(base, twl, tl);
    C wct[8];
    stages<0, DIR, PAR, ZM>(d, lds, twl, tl, no_xchg, base, fill, tw1, wct);
  }
  // IFFT then FFT of one antenna / CNC iteration: an even number of exchanges in total.
  template <int DIR, typename Fill = NoFill>
  static __device__ __forceinline__ void run_second(C (&d)[P], C* lds, const C* __restrict__ tw, int t,
                                                    bool no_xchg = false, const Fill& fill = Fill{},
                                                    const C* tw1 = nullptr) {
    run<DIR, XCHG & 1, 0u, Fill>(d, lds, tw, t, no_xchg, fill, tw1);
  }
};

}  // namespace mimo
