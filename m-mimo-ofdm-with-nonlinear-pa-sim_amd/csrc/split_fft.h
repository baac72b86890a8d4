// Split team FFT for the fp64 F = 8192 instance (gfx950): one 512-thread team, 16 points
// per thread (trial_launch.h team_size64), same contract as TeamFft (team_fft.h) --
// un-normalised transforms, run<+1> = frequency -> time, run_second<-1> = time -> frequency,
// a pointwise step (the PA) between them -- but two LDS exchanges per transform instead of
// three (the exchanges are what the one-team-per-CU instance cannot
// overlap).
//
// Thread t = 64 w + 32 g + l (wave w, lane half g, l < 32) works on sub-transform g as
// virtual thread vt = 32 w + l of a 4096-point TeamFft over 256 threads (16 x 16 x 16, two
// exchanges through its own half of the LDS; both halves share every barrier).
//   frequency layout: bin 2 (vt + 256 m) + g at register m, i.e. cyclic in the frequency
//     thread tau = 2 vt + g (freq_thread; the kernel's slot map runs on tau);
//   inverse: the even bins' IDFT E (g = 0) and the odd bins' O (g = 1), then
//     x[n] = E[n] + e^{+j 2pi n / F} O[n], x[n + F/2] = E[n] - e^{+j 2pi n / F} O[n];
//   forward: A[n] = x[n] + x[n + F/2], B[n] = (x[n] - x[n + F/2]) e^{-j 2pi n / F}, the even
//     bins = DFT(A) (g = 0), the odd bins = DFT(B) (g = 1).
// The radix-2 operands E[n], O[n] (and x[n], x[n + F/2]) live in lanes l and l + 32 of one
// wave, register m: v_permlane32_swap (lanes 32-63 of vdst <-> lanes 0-31 of src) on the
// register pair (m, m + 8) brings both into one lane -- lanes < 32 then hold n = vt + 256 m,
// lanes >= 32 n = vt + 256 (m + 8) -- and the same swap after the forward radix-2 stage
// hands A to the low and B to the high lane half.  32 swaps per transform (4 dwords per
// fp64 complex pair) instead of one 128 KiB LDS round trip.
// Twiddles: the sub-transform's table (fft_tw_total(F/2, P) stage entries + its cot-tan
// region), then (cos a, tan a), a = -2 pi n / F for n < F/2 (the radix-2 stage, bfly_ct form).
// tests/test_fft_split.py restates the layout and the butterflies lane by lane.
#pragma once
#include "team_fft.h"

namespace mimo {

// (MIMO_SPLIT_FFT / MIMO_SPLIT_CT: tuning.h)
constexpr bool kSplitCt = MIMO_SPLIT_CT != 0;  // the sub-transforms' stages in cot-tan form
constexpr bool split_fft_used(int F, int T, bool f64) { return MIMO_SPLIT_FFT != 0 && f64 && F == 8192 && T == 512; }
// table layout (engine.hip split_twiddles)
constexpr int split_fft_r2_off(int F, int T) {
  return fft_tw_total(F / 2, F / T) + (kSplitCt ? fft_ct_n(F / 2, F / T) : 0);
}
constexpr int split_fft_tw_total(int F, int T) { return split_fft_r2_off(F, T) + F / 2; }

template <int F, int T, int NBUF, typename Re>
struct SplitFft {
  using C = cx<Re>;
  static constexpr int P = F / T;
  static constexpr int TH = T / 2;
  using Sub = TeamFft<F / 2, TH, NBUF, Re, false, false, false, kSplitCt>;
  static_assert(Sub::P == P && P % 2 == 0 && T % 64 == 0, "split plan: same points per thread");
  static_assert(!kSplitCt || Sub::CT_N == fft_ct_n(F / 2, P), "cot-tan table layout");
  static constexpr int LDS_TOTAL = 2 * Sub::LDS_TOTAL;
  static constexpr int XCHG = Sub::XCHG;  // exchange windows per transform (fill calls)
  static constexpr int R2_OFF = split_fft_r2_off(F, T);
  using NoFill = typename Sub::NoFill;

  static __device__ __forceinline__ int vthread(int t) { return ((t >> 6) << 5) | (t & 31); }
  static __device__ __forceinline__ int group(int t) { return (t >> 5) & 1; }
  static __device__ __forceinline__ int freq_thread(int t) { return (vthread(t) << 1) | group(t); }

  // lanes 32-63 of a <-> lanes 0-31 of b (both 64-bit components)
  static __device__ __forceinline__ void swap32(Re& a, Re& b) {
    static_assert(sizeof(Re) == 8, "fp64 instance");
    const uint64_t ua = __builtin_bit_cast(uint64_t, a), ub = __builtin_bit_cast(uint64_t, b);
    const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)ua, (uint32_t)ub, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(ua >> 32), (uint32_t)(ub >> 32), false, false);
    a = __builtin_bit_cast(Re, ((uint64_t)(uint32_t)hi[0] << 32) | (uint32_t)lo[0]);
    b = __builtin_bit_cast(Re, ((uint64_t)(uint32_t)hi[1] << 32) | (uint32_t)lo[1]);
  }
  static __device__ __forceinline__ void swap_halves(C (&d)[P]) {
#pragma unroll
    for (int m = 0; m < P / 2; ++m) {
      swap32(d[m].x, d[m + P / 2].x);
      swap32(d[m].y, d[m + P / 2].y);
    }
  }
  // (cos, tan) of the radix-2 twiddle of register pair m: n = vt + TH (m + P/2 g) (uniform
  // table base + a 32-bit lane offset: scalar-base loads, no 64-bit address arithmetic)
  static __device__ __forceinline__ C r2(const C* tw, int n0, int m) { return Sub::gload(tw + R2_OFF, n0 + TH * m); }

  template <int DIR, int PAR = 0, uint32_t ZM = 0, typename Fill = NoFill>
  static __device__ __forceinline__ void run(C (&d)[P], C* lds, const C* __restrict__ tw, int t,
                                             bool no_xchg = false, const Fill& fill = Fill{},
                                             const C* tw1 = nullptr) {
    static_assert(DIR == +1, "run: the inverse (frequency -> time) transform");
    (void)tw1;
    const C* twl = tw;
    int tl = t;
    asm volatile("" : "+s"(twl));
    asm volatile("" : "+v"(tl));
    const int vt = vthread(tl), g = group(tl);
    Sub::template run<DIR, PAR, ZM>(d, lds + g * Sub::LDS_TOTAL, twl, vt, no_xchg, fill, nullptr);
    C z[P / 2];
#pragma unroll
    for (int m = 0; m < P / 2; ++m) z[m] = r2(twl, vt + TH * (P / 2) * g, m);
    swap_halves(d);  // lanes < 32: (E, O) at n = vt + TH m; lanes >= 32: at vt + TH (m + P/2)
#pragma unroll
    for (int m = 0; m < P / 2; ++m) bfly_ct<DIR, false>(d[m], d[m + P / 2], z[m], d[m], d[m + P / 2]);
  }

  // Time (as run() leaves it: x[n] in d[m], x[n + F/2] in d[m + P/2]) -> frequency.
  template <int DIR, typename Fill = NoFill>
  static __device__ __forceinline__ void run_second(C (&d)[P], C* lds, const C* __restrict__ tw, int t,
                                                    bool no_xchg = false, const Fill& fill = Fill{},
                                                    const C* tw1 = nullptr) {
    static_assert(DIR == -1, "run_second: the forward (time -> frequency) transform");
    (void)tw1;
    const C* twl = tw;
    int tl = t;
    asm volatile("" : "+s"(twl));
    asm volatile("" : "+v"(tl));
    const int vt = vthread(tl), g = group(tl);
#pragma unroll
    for (int m = 0; m < P / 2; ++m) {
      const C z = r2(twl, vt + TH * (P / 2) * g, m);  // forward: e^{-j 2pi n / F} = c (1 + j t)
      const C a = d[m], b = d[m + P / 2];
      const C u = csub(a, b);
      d[m] = cadd(a, b);
      d[m + P / 2] = mkc(z.x * fmar(-z.y, u.y, u.x), z.x * fmar(z.y, u.x, u.y));
    }
    swap_halves(d);  // lanes < 32: A at n = vt + TH m (all m); lanes >= 32: B
    Sub::template run_second<DIR>(d, lds + g * Sub::LDS_TOTAL, twl, vt, no_xchg, fill, nullptr);
  }
};

}  // namespace mimo
