// Wave-split team FFT for the fused trial kernel (gfx950; the instances wave_fft_used() names).
//
// Same contract as TeamFft (team_fft.h): T threads, P = F / T points per thread, the
// frequency-domain vector in the CYCLIC layout (bin e at thread e % T, register e / T),
// un-normalised transforms, run<+1> = frequency -> time, run_second<-1> = time ->
// frequency.  Only the time-domain layout differs, and the PA between the two
// transforms is pointwise.
//
// Four-step split F = WV x FW over the team's WV = T / 64 waves (FW = 64 P):
//   bin k = n2 + FW n1, time n = k1 + WV k2 (n2, k2 < FW; n1, k1 < WV)
//   inverse:  A[k1, n2] = sum_n1 X[n2 + FW n1] e^{+j 2pi n1 k1 / WV}    (in registers)
//             A'        = A e^{+j 2pi k1 n2 / F}
//             x[k1 + WV k2] = sum_n2 A'[k1, n2] e^{+j 2pi n2 k2 / FW}  (wave k1, one wave)
//   forward:  the mirror image (the wave-local FW-point transforms first).
// Thread t holds n2 = t + T i (i < NB = P / WV) for every n1: registers i + NB n1 of the
// cyclic layout.  The radix-WV step is the only one that crosses waves; the FW-point
// transforms (TeamFft<FW, 64, WAVE>) exchange through the wave's own LDS row with no
// hardware barrier.  One s_barrier per transform instead of one or two per exchange.
//
// LDS: WV rows of TeamFft<FW, 64>::LDS_ELEMS (the wave-local exchanges' padded buffer);
// the cross-wave step uses row k1 / row w unpadded.  Thread t writes and reads only the
// cross-wave cells [row][t + T i], so the next transform's cross-wave write needs no
// barrier before it (each thread rewrites exactly the cells it read itself), and a wave's
// row is touched by other waves only inside the cross-wave step, which the barrier
// brackets.
//
// Twiddle table (engine.hip): TeamFft<FW, 64>'s stage blocks, then exp(-j 2pi n / F) for
// n < F (the inter-step twiddles, exponents up to (WV - 1)(FW - 1)).
#pragma once
#include "team_fft.h"

namespace mimo {

// The plan needs at least two waves and whole radix-WV butterflies per thread.
constexpr bool wave_fft_ok(int F, int T) {
  return T >= 128 && T % 64 == 0 && (F / T) >= (T / 64) && (F / T) % (T / 64) == 0;
}
// Instances that use it (kernel and engine): fp64 up to F = 2048.  fp32: not used (F = 8192's 8-wave
// teams measured 17.43 -> 17.64 ms with it, profiles/r02/ab/ab_wavefft_8192_f32.json; below
// F = 8192 the 2-wave fp32 teams need only two exchanges per transform, which the split
// would raise to three).
// fp64 config 2: 58.82 -> 58.50 ms (profiles/r02/ab/ab_wavefft_2048_f64.json).  The
// barriers were not what the exchanges cost: their LDS round trips remain.
constexpr bool wave_fft_used(int F, int T, bool f64) {
  // F 4096 / 8192 run 16-point teams (trial_launch.h team_size64) on the team FFT: the
  // wave-split rows would not leave room for a second team at F 4096, and measured
  // neutral at F 8192 (profiles/r03/ab8k/ab_p16_wave.json).
  return wave_fft_ok(F, T) && f64 && F <= 2048;
}
constexpr int wave_fft_fw(int F, int T) { return F / (T / 64); }
constexpr int wave_fft_tw_inter(int F, int T) { return fft_tw_total(wave_fft_fw(F, T), F / T); }
constexpr int wave_fft_tw_total(int F, int T) { return wave_fft_tw_inter(F, T) + F; }
// The fp64 sub-transforms' cot-tan constants (team_fft.h dft8_ct) follow the inter twiddles
// (fft_ct_n entries).
constexpr int wave_fft_ct_n(int F, int T) { return fft_ct_n(wave_fft_fw(F, T), F / T); }

template <int F, int T, typename Re, bool LTW1 = true, bool LTW2 = LTW1>
struct WaveFft {
  using C = cx<Re>;
  static constexpr int P = F / T;
  static constexpr int WV = T / 64;
  static constexpr int FW = F / WV;
  static constexpr int NB = P / WV;
  static_assert(wave_fft_ok(F, T), "wave-split plan needs >= 2 waves and P a multiple of the wave count");
  // LTW1: stage-1 twiddles from LDS (tw1); from four waves on (F 2048) also stage 2's rows
  // r = 3, 5, 6 (config 2 -0.5 %, LoS -0.8 %, MCNC -1.0 %, profiles/r03/ab_x; at F 1024 the
  // 3 KiB more would cost the third wave per SIMD)
  // fp64 with both LDS twiddle blocks: the twiddled radix-8 stages absorb their twiddles
  // into FMAs (team_fft.h dft8_ct; the constants from the cot-tan region of the table)
  using Sub = TeamFft<FW, 64, 1, Re, true, LTW1, LTW2 && (T / 64) >= 4, sizeof(Re) == 8>;
  static constexpr int TW1_N = Sub::TW1_N;
  static constexpr int TWL_N = Sub::TWL_N;         // tw1: LDS copy of the entries twl_src names
  static __device__ __forceinline__ int twl_src(int i) {
    return Sub::CT ? wave_fft_tw_total(F, T) + i : Sub::twl_src(i);
  }
  static_assert(!Sub::CT || Sub::CT_N == wave_fft_ct_n(F, T), "cot-tan table layout");
  static_assert(Sub::P == P, "sub-transform keeps the points per thread");
  static constexpr int ROW = Sub::LDS_ELEMS;
#ifdef MIMO_DIAG_ROWS2
  // Diagnostic builds only (wrong results): the waves share two exchange rows (row w & 1), so
  // the team's exchange LDS halves -- the occupancy A/B of 4 waves / SIMD at F 2048
  // (profiles/r06/w4/), every access in bounds
  static constexpr int LDS_TOTAL = 2 * ROW;
  static __device__ __forceinline__ int row_of(int w) { return (w & 1) * ROW; }
#else
  static constexpr int LDS_TOTAL = WV * ROW;
  static __device__ __forceinline__ int row_of(int w) { return w * ROW; }
#endif
  static constexpr int XCHG = 1 + Sub::XCHG;  // exchange windows per transform (fill calls)
  static constexpr int TW_INTER = wave_fft_tw_inter(F, T);

  using NoFill = typename Sub::NoFill;
  static __device__ __forceinline__ int freq_thread(int t) { return t; }  // cyclic in t

  // Zero mask of radix-WV butterfly i's inputs v[n1] = d[i + NB n1] from the register mask.
  static constexpr uint32_t bfly_mask(uint32_t zm, int i) {
    uint32_t m = 0;
    for (int n1 = 0; n1 < WV; ++n1) m |= ((zm >> (i + NB * n1)) & 1u) << n1;
    return m;
  }

  // w[k] = exp(-j 2pi k n / F), k = 1 .. WV-1: powers of two loaded, the rest as products.
  static __device__ __forceinline__ void inter_tw(C (&w)[WV], const C* __restrict__ tw, int n) {
#pragma unroll
    for (int k = 1; k < WV; ++k) {
      if ((k & (k - 1)) == 0) {
        w[k] = Sub::gload(tw + TW_INTER, k * n);
      } else {
        int hb = k;
        while (hb & (hb - 1)) hb &= hb - 1;
        w[k] = cmul(w[hb], w[k - hb]);
      }
    }
  }

  template <int I, int DIR, uint32_t ZM>
  static __device__ __forceinline__ void inv_butterfly(C (&d)[P], C* lds, const C* __restrict__ tw, int t,
                                                       bool no_xchg) {
    C v[WV];
#pragma unroll
    for (int n1 = 0; n1 < WV; ++n1) v[n1] = d[I + NB * n1];
    Dft<WV, DIR, bfly_mask(ZM, I)>::run(v);
    const int n2 = t + T * I;
    C w[WV];
    inter_tw(w, tw, n2);
#pragma unroll
    for (int k1 = 1; k1 < WV; ++k1) v[k1] = cmulc(v[k1], w[k1]);  // DIR = +1: e^{+j ...}
    if (no_xchg) {
#pragma unroll
      for (int k1 = 0; k1 < WV; ++k1) d[I + NB * k1] = v[k1];
    } else {
#pragma unroll
      for (int k1 = 0; k1 < WV; ++k1) lds[row_of(k1) + n2] = v[k1];
    }
  }
  template <int DIR, uint32_t ZM, int I = 0>
  static __device__ __forceinline__ void inv_butterflies(C (&d)[P], C* lds, const C* __restrict__ tw, int t,
                                                         bool no_xchg) {
    if constexpr (I < NB) {
      inv_butterfly<I, DIR, ZM>(d, lds, tw, t, no_xchg);
      inv_butterflies<DIR, ZM, I + 1>(d, lds, tw, t, no_xchg);
    }
  }

  // Frequency (cyclic) -> time (wave k1, lane l, register m: n = k1 + WV (l + 64 m)).
  template <int DIR, int PAR = 0, uint32_t ZM = 0, typename Fill = NoFill>
  static __device__ __forceinline__ void run(C (&d)[P], C* lds, const C* __restrict__ tw, int t,
                                             bool no_xchg = false, const Fill& fill = Fill{},
                                             const C* tw1 = nullptr) {
    static_assert(DIR == +1, "run: the inverse (frequency -> time) transform");
    const C* twl = tw;
    int tl = t;
    asm volatile("" : "+s"(twl));
    asm volatile("" : "+v"(tl));
    inv_butterflies<DIR, ZM>(d, lds, twl, tl, no_xchg);
    const int w = tl >> 6, l = tl & 63;
    if (!no_xchg) {
      __syncthreads();
      const C* rb = lds + row_of(w) + l;
#pragma unroll
      for (int m = 0; m < P; ++m) d[m] = rb[64 * m];
    }
    fill(0);
    auto sub_fill = [&](int s) __attribute__((always_inline)) { fill(s + 1); };
    Sub::template run<DIR, 0, 0u>(d, lds + row_of(w), twl, l, no_xchg, sub_fill, tw1);
  }

  // Time (as run() leaves it) -> frequency (cyclic).
  template <int DIR, typename Fill = NoFill>
  static __device__ __forceinline__ void run_second(C (&d)[P], C* lds, const C* __restrict__ tw, int t,
                                                    bool no_xchg = false, const Fill& fill = Fill{},
                                                    const C* tw1 = nullptr) {
    static_assert(DIR == -1, "run_second: the forward (time -> frequency) transform");
    const C* twl = tw;
    int tl = t;
    asm volatile("" : "+s"(twl));
    asm volatile("" : "+v"(tl));
    const int w = tl >> 6, l = tl & 63;
    Sub::template run<DIR, 0, 0u>(d, lds + row_of(w), twl, l, no_xchg, fill, tw1);
    // B'[w, q] = B[w, q] e^{-j 2pi w q / F}, q = l + 64 m (wave-uniform branch)
    // (all P loads issued before the first multiply: one wait instead of P round trips).
    // The products go straight to the exchange row inside the branch: merged back into d
    // after it, they cost P register-pair copies per transform (v_mov_b64 at the join).
    C* wb = lds + row_of(w) + l;
    if (w > 0) {
      C tw[P];
#pragma unroll
      for (int m = 0; m < P; ++m) tw[m] = Sub::gload(twl + TW_INTER, w * (l + 64 * m));
      if (no_xchg) {
#pragma unroll
        for (int m = 0; m < P; ++m) d[m] = cmul(d[m], tw[m]);
      } else {
#pragma unroll
        for (int m = 0; m < P; ++m) wb[64 * m] = cmul(d[m], tw[m]);
      }
    } else if (!no_xchg) {
#pragma unroll
      for (int m = 0; m < P; ++m) wb[64 * m] = d[m];
    }
    if (!no_xchg) __syncthreads();
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      C v[WV];
#pragma unroll
      for (int w2 = 0; w2 < WV; ++w2) v[w2] = no_xchg ? d[i + NB * w2] : lds[row_of(w2) + tl + T * i];
      Dft<WV, DIR>::run(v);
#pragma unroll
      for (int k1 = 0; k1 < WV; ++k1) d[i + NB * k1] = v[k1];
    }
    fill(Sub::XCHG);
  }
};

}  // namespace mimo
