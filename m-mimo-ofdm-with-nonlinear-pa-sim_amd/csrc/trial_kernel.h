// Fused Monte-Carlo BER trial kernel for gfx950 (MI355X).
//
// One workgroup ("team", T threads) runs one trial = one OFDM symbol of
// mp_model.Link.simulate (mp_model.py:180-222; clean run :133-175) entirely on chip:
//
//   labels (Philox BITS) -> pre-weighted symbols s / ||H|| / sqrt(F) (LDS)   mp_model.py:208
//   pass 1: channel power draws -> MRT norms sum_a |H|^2   antenna_array.py:162-173
//           (Rayleigh: rho^2 = -ln u1 only, no sqrt / sin / cos)
//   pass 3: per antenna a
//       H (Philox CHAN x FSPL, or closed-form LoS/two-path)  channel.py:35-72,116-167,262-275
//       alpha_a from the per-antenna precoding power      mp_model.py:312-326
//       X = s conj(H) / ||H||  -> IFFT -> PA -> FFT       modulation.py:332-361, distortion.py, utilities.py:311-329
//       r += H Y,  g += alpha_a |H|^2 / ||H||             channel.py:287-290, mp_model.py:320-326
//   AWGN (Philox NOISE) scaled by Es eta / snr, z = (r + n)/g   noise.py:56-83, mp_model.py:210-214
//   CNC (corrector.py:52-112) or MCNC (corrector.py:165-207) iterations, hard slicer,
//   XOR-popcount bit errors -> counts[trial][idx]         mp_model.py:215-222
//
// Nothing per trial touches HBM except the final per-trial counts (n_idx x 4 B) and the
// receiver stage's register spills: the channel is regenerated from Philox instead of
// being stored.  Frequency-domain data live in the team FFT's cyclic
// register layout; each thread owns NSLOT in-band sub-carriers ("slots").
//
// Without CSI errors the per-sub-carrier FSPL ratio f_c/f_k is factored out of the
// antenna loops (it cancels in MRT) and the per-antenna ratio is folded into the
// Box-Muller radius; alpha_a comes from a host-fitted polynomial (fp32, F <= 4096) or a
// Chebyshev series (fp64).  Both instances are VALU-issue-bound.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "tuning.h"
#include "alpha_fit.h"
#include "philox.h"
#include "team_fft.h"
#include "wave_fft.h"
#include "split_fft.h"

namespace mimo {

enum PaKind : int { PA_NONE = 0, PA_SOFTLIM = 1, PA_RAPP = 2, PA_TOI = 3 };
enum ChanKind : int { CH_RAYLEIGH = 1, CH_LOS = 2, CH_TWOPATH = 3, CH_TABLE = 4 };
enum RxKind : int { RX_CNC = 1, RX_MCNC = 2 };

constexpr int kMaxCsiAnt = 512;  // CSI-error runs: antennas (dynamic LDS per team, A doubles; engine.hip checks)
constexpr uint32_t kFixedCsiTrial = 0xFFFFFFFFu;  // CSI stream counter of fixed-channel runs (oracle/sim.py draws)
// The measured alternatives of the choices below (channel pipeline on / off per precision,
// register diet from F 8192, raw-word pipeline, alpha by library exp / erfc, shfl vs DPP
// sums) are in DESIGN.md §3 and profiles/r02/ab/; the losing variants were removed.

template <typename R>
struct TrialParams {
  using C = cx<R>;
  uint64_t seed;
  uint64_t first_trial;
  uint32_t* counts;              // [n_trials][n_idx]
  const C* tw;                   // team-FFT stage twiddles of (F, T) (team_fft.h fft_tw_off)
  const C* tw_wave;              // wave-split FFT twiddles of (F, T) (wave_fft.h), or null
  const R* ant_rel;              // [A]  d0 / d_a      (Rayleigh FSPL, relative)
  const R* f_rel;                // [S]  fc / f_k      (f_k float32-quantised as in the reference)
  const double* f_over_c;        // [S]  f_k / c       (LoS / two-path phases)
  const double* tx_pos;          // [A*3]
  const double2* lut;            // [kLut64] fp64 ln / sincos tables (real.h; fp64 instances only)
  const C* chan_tab;             // CH_TABLE: fixed in-band channel [A][S] (sub-carrier order k)
  int n_ant, n_sc, qam_l, half_bits;
  uint32_t label_mask;
  int pa_kind, cnc_pa_kind;
  R sat_tx, sqrt_sat_tx, inv_sat_tx, rapp_p, toi_tx;
  R sat_cnc, sqrt_sat_cnc, inv_sat_cnc, toi_cnc, inv_alpha_cnc;
  R alpha_c;                     // 10^(IBO/10) S / A : gamma_a^2 = alpha_c / vk_pow[a]
  // alpha(gamma_a^2) as a degree-8 polynomial in x = vk_pow[a] A / S - 1 on |x| <= alpha_xlim
  // (host Chebyshev fit, ~1e-7 relative); the exact formula outside (engine.hip fit_alpha).
  // fp32 instances only: the fp64 instances always evaluate the exact formula.
  R apoly[9];
  R inv_vk0, alpha_xlim;
  R inv_vk0_f;                   // inv_vk0 F (the fp64 register-diet array pass sums vk / F)
  // fp64 instances: alpha(gamma_a^2) as a degree-18 polynomial in x on |x| <= alpha_xlim
  // (the host's Chebyshev interpolant at 64 nodes in long double, as monomials: Horner,
  // <= 1.6e-16 relative; the singularity of alpha(g0^2 / (1 + x)) at x = -1 is 4
  // half-widths away), the exact formula outside.
  double amono64[19];
  R es_over_snr;                 // Es / 10^(SNR/10)
  R csi_a, csi_b;                // sqrt(1 - eps^2), eps
  R inv_sqrt_f;
  int receiver;
  int max_iter;                  // largest iteration index to run (CNC / MCNC)
  uint32_t rec_mask;             // bit i: record iteration i
  int incl_clean, n_idx;
  double rx_x0, rx_z, rx_var, d0; // LoS / two-path geometry
  uint32_t ablate;               // diagnostic builds only (-DMIMO_ABLATION), see ABL_* below
  // Multi-point launches (mimo_engine_run_points): the kernel argument carries the table;
  // block b runs trial points[i].first_trial + b - point_start[i] of point i, where
  // point_start[i] <= b < point_start[i + 1].  The per-point parameters (PA, AGC, noise,
  // seed ...) are read from points[i] through the constant address space (scalar loads).
  const TrialParams* points;     // [n_points] (device)
  const uint32_t* point_start;   // [n_points + 1] block offsets (device)
  int n_points;
  uint32_t chan_period;          // 0, or the channel-replay period (mimo_config.chan_replay_period)
  // Last, so that the fields the antenna loop reloads keep their 16-byte alignment (the
  // scalar loads pair them as s_load_dwordx4; inserted after `seed` it cost the F 4096
  // instance 1 %, profiles/r04/misc/).
  uint64_t csi_seed;             // CH_TABLE + CSI: key of the one shared estimate (mimo_config.csi_seed)
};

// Ablation switches for cost breakdowns.  Compiled in only with -DMIMO_ABLATION
// (libmimo_engine_ablation.so); the production kernel has none of these branches.
enum : uint32_t { ABL_RNG = 1, ABL_FFT = 2, ABL_PASS1 = 4, ABL_PA = 8, ABL_XCHG = 16 };
// ISA inspection only (tools/stage_hist.py): a comment in the assembly naming the loop.
#ifdef MIMO_ISA_MARKERS
#define MIMO_ISA_MARK(name) asm volatile("; MIMO_MARK " name)
#else
#define MIMO_ISA_MARK(name) ((void)0)
#endif
#ifdef MIMO_ABLATION
#define MIMO_ABL(p, bit) (((p).ablate & (bit)) != 0)
#elif defined(MIMO_STATIC_ABLATE)  // ISA inspection only (tools/stage_hist.py): stages compiled out
#define MIMO_ABL(p, bit) ((MIMO_STATIC_ABLATE & (bit)) != 0)
#else
#define MIMO_ABL(p, bit) false
#endif

// ---------------------------------------------------------------- slot geometry
// ALIGNED: S % (4T) == 0 and S < F.  Slot s < HALF is the positive band (bin
// n = t + T s, k = n + S/2 - 1; thread 0 slot 0 is bin S/2 instead of DC); slot s >= HALF
// is the negative band (bin F - S/2 + t + T (s - HALF), k = t + T (s - HALF)).
// Generic: slot s = register s, valid iff its bin is in band.
template <int F, int T, int NSLOT, bool ALIGNED>
struct Slots {
  static constexpr int P = F / T;
  static constexpr int HALF = NSLOT / 2;
  static constexpr int m_of(int s) { return ALIGNED ? (s < HALF ? s : P - NSLOT + s) : s; }
  // Registers the scatter leaves zero in every thread: the out-of-band middle
  // (HALF + 1 .. P - HALF - 1; register HALF holds thread 0's bin S/2).  Generic: none.
  static constexpr uint32_t zero_mask() {
    uint32_t m = 0;
    if (ALIGNED)
      for (int r = HALF + 1; r < P - HALF; ++r) m |= 1u << r;
    return m;
  }

  static __device__ __forceinline__ int k_of(int s, int t, int S, bool& valid) {
    if constexpr (ALIGNED) {
      valid = true;
      if (s < HALF) {
        const int n = (s == 0 && t == 0) ? (S >> 1) : t + T * s;
        return n + (S >> 1) - 1;
      }
      return t + T * (s - HALF);
    } else {
      const int n = t + T * s;
      const int lo = F - (S >> 1);
      valid = (n >= 1 && n <= (S >> 1)) || n >= lo;
      return !valid ? 0 : (n >= lo ? n - lo : n + (S >> 1) - 1);  // 0 keeps table reads in bounds
    }
  }

  template <class C>
  static __device__ __forceinline__ void scatter(C (&d)[P], const C (&x)[NSLOT], bool t0) {
    using R = real_of<C>;
#pragma unroll
    for (int m = 0; m < P; ++m) d[m] = czero<R>();
#pragma unroll
    for (int s = 0; s < NSLOT; ++s) {
      if constexpr (ALIGNED) {
        if (s == 0) {
          // thread 0's slot 0 is bin S/2 (register HALF), the others' bin t (register 0):
          // two multiplies by 0 / 1 per component instead of four 32-bit selects
          const R m1 = t0 ? R(1) : R(0), m0 = R(1) - m1;
          d[0] = cscale(x[0], m0);
          d[HALF] = cscale(x[0], m1);
          continue;
        }
      }
      d[m_of(s)] = x[s];
    }
  }

  template <class C>
  static __device__ __forceinline__ C gather(const C (&d)[P], int s, bool t0) {
    if constexpr (ALIGNED) {
      if (s == 0) return t0 ? d[HALF] : d[0];
    }
    return d[m_of(s)];
  }
};

// ---------------------------------------------------------------- small helpers
// Opaque copy: stops LICM from hoisting thread-invariant derived values (slot->k maps,
// Philox round-0 products, QAM points, table loads) out of the antenna loop, which
// would keep dozens of VGPRs live across it and spill.  Re-deriving them is cheap.
template <typename V>
__device__ __forceinline__ V opaque(V v) {
  asm volatile("" : "+v"(v));
  return v;
}
template <typename R>
__device__ __forceinline__ R wave_sum(R v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Wave sum delivered in lane 63 only (other lanes hold partial sums): DPP adds on the
// VALU instead of the six dependent ds_bpermute round trips of __shfl_xor.  Per row of
// 16 lanes: pair / quad swaps and the half-row / row mirrors give every lane its row sum;
// row_bcast:15 then row_bcast:31 fold rows 0-2 into row 3.  (fp64: both halves moved.)
// mov_dpp leaves the lanes of disabled rows undefined (no zero-initialised "old" operand,
// one v_mov fewer per step): after the row_bcast:15 step rows 0 and 2 hold garbage, which
// no later step reads (row_bcast:31 reads lane 31, row 1) and lane 63 never sees.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ float dpp_add(float v) {
  const int s = __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, ROW_MASK, 0xF, false);
  return v + __builtin_bit_cast(float, s);
}
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ double dpp_add(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)u, CTRL, ROW_MASK, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), CTRL, ROW_MASK, 0xF, false);
  return v + __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
template <typename R>
__device__ __forceinline__ R wave_sum_lane63(R v) {
  v = dpp_add<0xB1>(v);        // quad_perm [1,0,3,2]
  v = dpp_add<0x4E>(v);        // quad_perm [2,3,0,1]
  v = dpp_add<0x141>(v);       // row_half_mirror
  v = dpp_add<0x140>(v);       // row_mirror
  v = dpp_add<0x142, 0xA>(v);  // row_bcast:15 into rows 1 and 3
  v = dpp_add<0x143, 0xC>(v);  // row_bcast:31 into rows 2 and 3
  return v;
}

// Team-wide sum; every thread gets the result.  Two barriers.
template <int T, typename R>
__device__ __forceinline__ R team_sum(R v, R* red) {
  if constexpr (T == 64) {
    return wave_sum(v);
  } else {
    v = wave_sum_lane63(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 63) red[threadIdx.x >> 6] = v;
    __syncthreads();
    R s = R(0);
#pragma unroll
    for (int i = 0; i < T / 64; ++i) s += red[i];
    return s;
  }
}

// Bussgang gain, modulation.py:178-189, from gamma^2.
__device__ __forceinline__ float alpha_of_gamma2(float g2) {
  const float g = __builtin_sqrtf(g2);
  return 1.0f - __expf(-g2) + 0.88622692545275801f * g * erfcf(g);
}
__device__ __forceinline__ double alpha_of_gamma2(double g2) {
  const double g = __builtin_sqrt(g2);
  return 1.0 - exp(-g2) + 0.88622692545275801 * g * erfc(g);
}

// PA on one time-domain sample (distortion.py:9-19, 102-113, 202-211).
// Soft limiter: min(1, sqrt(sat) rsq(pw)) -- the reference's branch |x|^2 > sat, then
// x sqrt(sat / |x|^2), up to rounding at |x|^2 = sat (fp64: -0.4 % against the branch).
template <class C, typename R = real_of<C>>
__device__ __forceinline__ C pa_apply(int kind, C x, R sat, R sqrt_sat, R inv_sat, R rapp_p, R toi) {
  const R pw = fmar(x.x, x.x, x.y * x.y);
  R sc = R(1);
  if (kind == PA_SOFTLIM) {
    if constexpr (sizeof(R) == 4) sc = minr(1.0f, sqrt_sat * rsq_r(pw));
    else sc = fmin(R(1), sqrt_sat * rsq_n1(pw));  // rsq(0) = inf -> NaN -> fmin picks 1
  } else if (kind == PA_RAPP) {
    // 1 / (1 + (pw/sat)^p)^(1/(2p))
    const R u = pw * inv_sat;
    const R up = u > R(0) ? exp2_r(rapp_p * log2_r(u)) : R(0);
    sc = exp2_r(-(R(0.5) / rapp_p) * log2_r(R(1) + up));
  } else if (kind == PA_TOI) {
    sc = R(1) - toi * pw;
  }
  return mkc(x.x * sc, x.y * sc);
}

// Cold path out of line: the general-hardness Rapp gain (library log2 / exp2).  Inlined,
// its f64 constants were hoisted into the loop preheader and spilled to scratch once per
// trial (~90 KB of writes per trial at config 2, profiles/r03/pmc); out of line they stay
// in the call.  Measured with the exact-alpha fallback (now alpha_fit.h's segment table,
// which has no constants to hoist) outlined as well: config 2 -2.5 %, CSI -2.7 %, LoS
// -2.3 %, two-path -3.0 %, F 8192 -0.4 %; F 4096 +1.6 % (profiles/r03/ab_s/).
template <class C, typename R = real_of<C>>
__device__ __attribute__((noinline)) C pa_rapp_general(C x, R inv_sat, R rapp_p) {
  return pa_apply(PA_RAPP, x, R(0), R(0), inv_sat, rapp_p, R(0));
}

// y^(-1/N) for y >= 1 (the Rapp gain at integer hardness, N = 2p).  fp32: hardware
// log / exp.  fp64: the fp32 hardware value z as the seed (~2^-22) and one third-order
// step z (1 - e)^(-1/N) ~ z (1 + e/N + (N+1) e^2 / (2 N^2)), e = 1 - y z^N (error
// ~2^-60, below the fp64 rounding): 7 f64 ops + 2 fp32 transcendentals instead of the
// library log2 + exp2 (~60 instructions).
template <int N>
__device__ __forceinline__ float rpow_neg_inv(float y) {
  return __builtin_amdgcn_exp2f((-1.0f / N) * __builtin_amdgcn_logf(y));
}
template <int N>
__device__ __forceinline__ double rpow_neg_inv(double y) {
  static_assert(N == 4 || N == 6, "integer Rapp hardness 2 or 3");
  const double z = (double)rpow_neg_inv<N>((float)y);
  const double z2 = z * z;
  const double zn = N == 4 ? z2 * z2 : z2 * z2 * z2;
  const double e = fma(-y, zn, 1.0);
  const double c = e * fma(e, (N + 1.0) / (2.0 * N * N), 1.0 / N);
  return fma(z, c, z);
}

// Rapp with an integer hardness: (pw/sat)^p by multiplication (config 5 uses p = 3), then
// (1 + (pw/sat)^p)^(-1/(2p)) by rpow_neg_inv.
template <int IP, int P, class C, typename R = real_of<C>>
__device__ __forceinline__ void rapp_int(C (&d)[P], R inv_sat) {
#pragma unroll
  for (int m = 0; m < P; ++m) {
    const R u = fmar(d[m].x, d[m].x, d[m].y * d[m].y) * inv_sat;
    R up = u;
#pragma unroll
    for (int i = 1; i < IP; ++i) up *= u;
    const R sc = rpow_neg_inv<2 * IP>(R(1) + up);
    d[m] = mkc(d[m].x * sc, d[m].y * sc);
  }
}

// PA on all P samples of a thread: one uniform branch on the kind, then a straight loop.
template <bool COLD_OUT, int P, class C, typename R = real_of<C>>
__device__ __forceinline__ void pa_block(int kind, C (&d)[P], R sat, R sqrt_sat, R inv_sat, R rapp_p, R toi) {
#ifdef MIMO_DIAG_PA_SOFTLIM_ONLY  // ISA inspection only (tools/one_inst.hip): no other PA kinds
  kind = PA_SOFTLIM;
#endif
  if (kind == PA_SOFTLIM) {
#pragma unroll
    for (int m = 0; m < P; ++m) d[m] = pa_apply(PA_SOFTLIM, d[m], sat, sqrt_sat, inv_sat, rapp_p, toi);
  } else if (kind == PA_RAPP && rapp_p == R(3)) {
    rapp_int<3>(d, inv_sat);
  } else if (kind == PA_RAPP && rapp_p == R(2)) {
    rapp_int<2>(d, inv_sat);
  } else if (kind == PA_RAPP) {
#pragma unroll
    for (int m = 0; m < P; ++m) {
      if constexpr (COLD_OUT) d[m] = pa_rapp_general(d[m], inv_sat, rapp_p);
      else d[m] = pa_apply(PA_RAPP, d[m], sat, sqrt_sat, inv_sat, rapp_p, toi);
    }
  } else if (kind == PA_TOI) {
#pragma unroll
    for (int m = 0; m < P; ++m) d[m] = pa_apply(PA_TOI, d[m], sat, sqrt_sat, inv_sat, rapp_p, toi);
  }
}

// Per-axis hard slicer == argmin |z - C| over the Gray-ordered constellation with the
// reference's first-index (lowest label) tie-break (modulation.py:75-76,138-146).
__device__ __forceinline__ uint32_t gray(uint32_t i) { return i ^ (i >> 1); }
__device__ __forceinline__ uint32_t gray_inv(uint32_t g) {
  g ^= g >> 1;
  g ^= g >> 2;
  g ^= g >> 4;
  g ^= g >> 8;
  return g;
}
template <typename R>
__device__ __forceinline__ uint32_t slice_axis(R x, int L) {
  const R q = (x + (R)L) * R(0.5);
  const R fi = floor_r(q);
  int i = (int)fi;
  if (q == fi && i > 0 && i < L) {  // exact midpoint between levels i-1 and i
    i = gray((uint32_t)(i - 1)) < gray((uint32_t)i) ? i - 1 : i;
  }
  i = i < 0 ? 0 : (i > L - 1 ? L - 1 : i);
  return gray((uint32_t)i);
}
template <class C>
__device__ __forceinline__ uint32_t slice(C z, int L, int hb) {
  return (slice_axis(z.x, L) << hb) | slice_axis(z.y, L);
}
template <typename R>
__device__ __forceinline__ cx<R> qam_point(uint32_t label, int L, int hb) {
  const uint32_t ii = gray_inv(label >> hb), iq = gray_inv(label & ((1u << hb) - 1u));
  return mkc((R)(2 * (int)ii - (L - 1)), (R)(2 * (int)iq - (L - 1)));
}
// The same point as two int16 lattice levels in one word (I high, Q low): the register
// diet keeps these per slot and rebuilds the point per antenna in 2 shifts + 2 converts
// instead of the two inverse Gray codes (~20 integer ops).
__device__ __forceinline__ uint32_t qam_levels(uint32_t label, int L, int hb) {
  const int ii = 2 * (int)gray_inv(label >> hb) - (L - 1), iq = 2 * (int)gray_inv(label & ((1u << hb) - 1u)) - (L - 1);
  return ((uint32_t)ii << 16) | ((uint32_t)iq & 0xFFFFu);
}
// Two slots per word for the register diet: int8 lattice levels (|level| <= L - 1 <= 63 for
// M <= 4096), slot 2 i + h in bits 16 h .. 16 h + 15 of word i (I high byte): half the VGPRs
// of one word per slot, and the same 2 extracts + 2 converts (v_bfe_i32) to rebuild.
__device__ __forceinline__ uint32_t qam_levels8(uint32_t label, int L, int hb) {
  const int ii = 2 * (int)gray_inv(label >> hb) - (L - 1), iq = 2 * (int)gray_inv(label & ((1u << hb) - 1u)) - (L - 1);
  return (((uint32_t)ii & 0xFFu) << 8) | ((uint32_t)iq & 0xFFu);
}
template <typename R, int H>
__device__ __forceinline__ cx<R> levels_point8(uint32_t w) {
  // sign-extending extracts of bits 16 H + 8 .. + 15 (I) and 16 H .. + 7 (Q)
  return mkc((R)((int)(w << (16 - 16 * H)) >> 24), (R)((int)(w << (24 - 16 * H)) >> 24));
}
template <typename R>
__device__ __forceinline__ cx<R> levels_point(uint32_t v) {
  return mkc((R)((int)v >> 16), (R)(int)(int16_t)(v & 0xFFFFu));
}

// ---------------------------------------------------------------- channel generation
// sin / cos of a channel phase in revolutions: fp32 hardware (v_sin / v_cos take
// revolutions), fp64 the table form (real.h sincos_rev_lut).
__device__ __forceinline__ void sincos_phase(float r, float& sn, float& cs) {
  sn = sin_rev(r);
  cs = cos_rev(r);
}
__device__ __forceinline__ void sincos_phase(double r, double& sn, double& cs) {
  sincos_rev_lut(r, sn, cs);
}

template <typename R, int F, int T, int NSLOT, bool ALIGNED, int CH, bool UNI_EXTRA = false>
struct Channel {
  // philox.h UNI rounds (the rounds whose words are uniform across the team on the SALU): the
  // fp64 wave-split instances (F <= 2048), and UNI_EXTRA (the F 4096 CSI instance, below)
  static constexpr bool kUni = sizeof(R) == 8 && (wave_fft_used(F, T, true) || UNI_EXTRA);
  using SL = Slots<F, T, NSLOT, ALIGNED>;
  using C = cx<R>;
  using Params = TrialParams<R>;

  // CN(0,1) draws of one stream for the thread's slots (pairs resolved in-thread when aligned).
  // c = bm_c(scale^2) scales the draws (box_muller).
  static __device__ __forceinline__ void normals(Key key, uint32_t trial, uint32_t stream, uint32_t aux, int t, int S,
                                                 C (&z)[NSLOT], R c = bm_c<R>(R(1))) {
    if constexpr (ALIGNED) {
      // Pair indices in closed form (pair_of() applied to the aligned slot map):
      //   positive band, slots j and j + Q: q = S/4 - 1 + t + T j, except thread 0 /
      //   j = 0 (bins S/2 and S/4): q = S/2 - 1 with the two draws swapped;
      //   negative band, slots HALF + j and HALF + j + Q: q = t + T j.
      constexpr int Q = SL::HALF / 2;
      const bool t0 = (t == 0);
      const int qp = (S >> 2) - 1 + t;
#pragma unroll
      for (int j = 0; j < Q; ++j) {
        C z1, z2;
        const bool sw = (j == 0) && t0;
        cn_pair<kUni>(key, sw ? (uint32_t)((S >> 1) - 1) : (uint32_t)(qp + T * j), trial, stream, aux, z1, z2, c, sw);
        z[j] = z1;
        z[j + Q] = z2;
        cn_pair<kUni>(key, (uint32_t)(t + T * j), trial, stream, aux, z1, z2, c);
        z[SL::HALF + j] = z1;
        z[SL::HALF + j + Q] = z2;
      }
    } else {
#pragma unroll
      for (int s = 0; s < NSLOT; ++s) {
        bool v;
        const int k = SL::k_of(s, t, S, v);
        z[s] = czero<R>();
        if (v) {
          uint32_t q;
          int slot;
          pair_of(k, S, q, slot);
          C z1, z2;
          cn_pair<kUni>(key, q, trial, stream, aux, z1, z2, c);
          z[s] = slot == 0 ? z1 : z2;
        }
      }
    }
  }

  // One Philox call's worth of normals() (aligned instances): chunk c = 2 j + band fills
  // slots (j, j + Q) of the positive band (band 0) or (HALF + j, HALF + j + Q) of the
  // negative band (band 1).  normals() == all 2 Q chunks.
  static constexpr int kChunks = ALIGNED ? SL::HALF : 0;
  static __device__ __forceinline__ void normals_chunk(int c, Key key, uint32_t trial, uint32_t stream, uint32_t aux,
                                                       int t, int S, C (&z)[NSLOT], R cs) {
    if constexpr (ALIGNED) {
      constexpr int Q = SL::HALF / 2;
      const int j = c >> 1;
      C z1, z2;
      if ((c & 1) == 0) {
        const bool sw = (j == 0) && (t == 0);
        cn_pair<kUni>(key, sw ? (uint32_t)((S >> 1) - 1) : (uint32_t)((S >> 2) - 1 + t + T * j), trial, stream, aux, z1, z2,
                cs, sw);
        z[j] = z1;
        z[j + Q] = z2;
      } else {
        cn_pair<kUni>(key, (uint32_t)(t + T * j), trial, stream, aux, z1, z2, cs);
        z[SL::HALF + j] = z1;
        z[SL::HALF + j + Q] = z2;
      }
    }
  }

  // |H|^2 of antenna a at the thread's slots (Rayleigh, FSPL factor f_rel left out as in
  // gen<false>): the same draws as gen(), magnitudes only.
  template <class PP>
  static __device__ __forceinline__ void power(const PP& p, Key key, uint32_t trial, int a, int t,
                                               R (&e2)[NSLOT]) {
    const int S = p.n_sc;
    const R sa = p.ant_rel[a];
    const R c = bm_c<R>(sa * sa);
    if constexpr (ALIGNED) {
      constexpr int Q = SL::HALF / 2;
      const bool t0 = (t == 0);
      const int qp = (S >> 2) - 1 + t;
#pragma unroll
      for (int j = 0; j < Q; ++j) {
        R p1, p2;
        const bool sw = (j == 0) && t0;
        cn_pair_pow<kUni>(key, sw ? (uint32_t)((S >> 1) - 1) : (uint32_t)(qp + T * j), trial, ST_CHAN, (uint32_t)a, p1, p2,
                    c, sw);
        e2[j] = p1;
        e2[j + Q] = p2;
        cn_pair_pow<kUni>(key, (uint32_t)(t + T * j), trial, ST_CHAN, (uint32_t)a, p1, p2, c);
        e2[SL::HALF + j] = p1;
        e2[SL::HALF + j + Q] = p2;
      }
    } else {
#pragma unroll
      for (int s = 0; s < NSLOT; ++s) {
        bool v;
        const int k = SL::k_of(s, t, S, v);
        e2[s] = R(0);
        if (v) {
          uint32_t q;
          int slot;
          pair_of(k, S, q, slot);
          R p1, p2;
          cn_pair_pow<kUni>(key, q, trial, ST_CHAN, (uint32_t)a, p1, p2, c);
          e2[s] = slot == 0 ? p1 : p2;
        }
      }
    }
  }

  // Polar form of normals() (aligned instances): rho^2 = c ln u1 and the angle word w1 of
  // every slot's draw (the draw is rho e^{j 2 pi w1 2^-32}, box_muller), no sqrt / sin / cos.
  // fn(slot, rho^2, angle word) per slot, one Philox call (two slots) at a time.
  template <class Fn>
  static __device__ __forceinline__ void polar(Key key, uint32_t trial, uint32_t stream, uint32_t aux, int t, int S, R c,
                                               const Fn& fn) {
    static_assert(ALIGNED, "aligned slot map");
    constexpr int Q = SL::HALF / 2;
    const bool t0 = (t == 0);
    const int qp = (S >> 2) - 1 + t;
#pragma unroll
    for (int j = 0; j < Q; ++j) {
      const bool sw = (j == 0) && t0;
      uint4 w = philox4x32_10<kUni>(make_uint4(sw ? (uint32_t)((S >> 1) - 1) : (uint32_t)(qp + T * j), trial, stream, aux),
                                    key);
      fn(j, c * bm_log(sw ? w.z : w.x, R(0)), sw ? w.w : w.y);
      fn(j + Q, c * bm_log(sw ? w.x : w.z, R(0)), sw ? w.y : w.w);
      w = philox4x32_10<kUni>(make_uint4((uint32_t)(t + T * j), trial, stream, aux), key);
      fn(SL::HALF + j, c * bm_log(w.x, R(0)), w.y);
      fn(SL::HALF + j + Q, c * bm_log(w.z, R(0)), w.w);
    }
  }

  // normals() with a per-slot scale folded into the Box-Muller radius: z = (rho w_s) e^{j phi}
  // and rw = rho w_s (aligned instances) -- one multiply per draw instead of two.
  static __device__ __forceinline__ void normals_w(Key key, uint32_t trial, uint32_t stream, uint32_t aux, int t, int S,
                                                   R c, const R (&w)[NSLOT], C (&z)[NSLOT], R (&rw)[NSLOT]) {
    static_assert(ALIGNED, "aligned slot map");
    constexpr int Q = SL::HALF / 2;
    const bool t0 = (t == 0);
    const int qp = (S >> 2) - 1 + t;
    auto draw = [&](int s, uint32_t w0, uint32_t w1) __attribute__((always_inline)) {
      rw[s] = sqrt_n1(c * bm_log(w0, R(0))) * w[s];
      R sn, cs;
      sincos_lut(w1, sn, cs);
      z[s] = mkc(rw[s] * cs, rw[s] * sn);
    };
#pragma unroll
    for (int j = 0; j < Q; ++j) {
      const bool sw = (j == 0) && t0;
      uint4 u = philox4x32_10<kUni>(make_uint4(sw ? (uint32_t)((S >> 1) - 1) : (uint32_t)(qp + T * j), trial, stream, aux),
                                    key);
      draw(j, sw ? u.z : u.x, sw ? u.w : u.y);
      draw(j + Q, sw ? u.x : u.z, sw ? u.y : u.w);
      u = philox4x32_10<kUni>(make_uint4((uint32_t)(t + T * j), trial, stream, aux), key);
      draw(SL::HALF + j, u.x, u.y);
      draw(SL::HALF + j + Q, u.z, u.w);
    }
  }

  // |H|^2 of antenna a at the thread's slots for the closed-form channels (gen<false>'s
  // magnitudes, for pass 1's MRT norms): LoS |a1 e^{j phi1}|^2 = a1^2 -- no phase at all;
  // two-path |a1 e^{j phi1} - a2 e^{j phi2}|^2 = (a1 - a2)^2 + 4 a1 a2 sin^2((phi1 - phi2) / 2)
  // -- one sine of the half path difference instead of two sine / cosine pairs, in the
  // cancellation-free form: a2 / a1 = d_los / d_sec is within ~1e-3 of 1 for the reference's
  // geometry, so at a reflection null (aligned across a ULA) the true value sits near
  // (a1 - a2)^2 ~ 1e-7 a1^2, below the rounding of a1^2 + a2^2 - 2 a1 a2 cos in fp32.  The
  // difference a1 - a2 is formed in fp64 and the half phase reduced to [-1/4, 1/4] rev first.
  template <class PP>
  static __device__ __forceinline__ void power_closed(const PP& p, int a, int t, const double (&rx)[3],
                                                      R (&e2)[NSLOT]) {
    static_assert(CH == CH_LOS || CH == CH_TWOPATH, "closed-form channels");
    const int S = p.n_sc;
    const double tx = p.tx_pos[3 * a], ty = p.tx_pos[3 * a + 1], tz = p.tx_pos[3 * a + 2];
    const double dx = tx - rx[0], dy = ty - rx[1], dz = tz - rx[2];
    const double d_los = sqrt(dx * dx + dy * dy + dz * dz);
    const R att_los = (R)(p.d0 / d_los);
    if constexpr (CH == CH_LOS) {
#pragma unroll
      for (int s = 0; s < NSLOT; ++s) {
        bool v;
        SL::k_of(s, t, S, v);
        e2[s] = v ? att_los * att_los : R(0);
      }
    } else {
      const double hz = tz + rx[2];
      const double d_sec = sqrt(dx * dx + dy * dy + hz * hz);
      const double g_sec = p.d0 / d_sec;
      const R d12 = (R)(p.d0 / d_los - g_sec);
      const R a4 = R(4) * att_los * (R)g_sec;
      const R d12sq = d12 * d12;
      const double dd = d_los - d_sec;
#pragma unroll
      for (int s = 0; s < NSLOT; ++s) {
        bool v;
        const int k = SL::k_of(s, t, S, v);
        R e = R(0);
        if (v) {
          double ph = dd * p.f_over_c[k];
          ph -= rint(ph);  // [-1/2, 1/2] rev: the half phase keeps its relative precision
          R sn, cs;
          sincos_phase((R)(0.5 * ph), sn, cs);
          e = fmar(a4 * sn, sn, d12sq);
        }
        e2[s] = e;
      }
    }
  }

  // True channel of antenna a at the thread's slots (relative scale: common factors
  // cancel in MRT, AGC and the SNR normalisation).  FREL = false leaves out the
  // per-sub-carrier FSPL factor fc/f_k, which the kernel then applies once per trial
  // (it cancels in the MRT precoder; see the kernel's AWGN step).
  template <bool FREL, class PP>
  static __device__ __forceinline__ void gen(const PP& p, Key key, uint32_t trial, int a, int t,
                                             const double (&rx)[3], C (&h)[NSLOT]) {
    const int S = p.n_sc;
    if constexpr (CH == CH_RAYLEIGH) {
      const R sa = p.ant_rel[a];
      if (MIMO_ABL(p, ABL_RNG)) {
#pragma unroll
        for (int s = 0; s < NSLOT; ++s)
          h[s] = mkc(sa + R(1e-3) * (R)((a + s + t) & 7), R(0.5) - R(1e-3) * (R)((a * s) & 3));
      } else {
        normals(key, trial, ST_CHAN, (uint32_t)a, t, S, h, bm_c<R>(sa * sa));  // ant_rel folded in
      }
      if constexpr (FREL) {
#pragma unroll
        for (int s = 0; s < NSLOT; ++s) {
          bool v;
          const int k = SL::k_of(s, t, S, v);
          h[s] = cscale(h[s], v ? p.f_rel[k] : R(0));
        }
      }
    } else if constexpr (CH == CH_TABLE) {
      // the caller's fixed channel (Link.simulate reroll_chan=False): coalesced loads of the
      // in-band row (f_rel is 1 for table engines: nothing is factored out)
#pragma unroll
      for (int s = 0; s < NSLOT; ++s) {
        bool v;
        const int k = SL::k_of(s, t, S, v);
        h[s] = v ? p.chan_tab[(size_t)a * S + k] : czero<R>();
      }
    } else {
      const double tx = p.tx_pos[3 * a], ty = p.tx_pos[3 * a + 1], tz = p.tx_pos[3 * a + 2];
      const double dx = tx - rx[0], dy = ty - rx[1], dz = tz - rx[2];
      const double d_los = sqrt(dx * dx + dy * dy + dz * dz);
      const R att_los = (R)(p.d0 / d_los);
      double d_sec = 0.0;
      R att_sec = R(0);
      if constexpr (CH == CH_TWOPATH) {
        // channel.py:138-147: elevation from the mirrored geometry, d_sec = tz/sin(el) +
        // rz/sin(el) with el = atan((tz + rz) / horiz), i.e. the mirrored path length
        // sqrt(horiz^2 + (tz + rz)^2) (no fp64 atan / sin; equal to ~1e-16 relative)
        const double hz = tz + rx[2];
        d_sec = sqrt(dx * dx + dy * dy + hz * hz);
        att_sec = (R)(p.d0 / d_sec);
      }
#pragma unroll
      for (int s = 0; s < NSLOT; ++s) {
        bool v;
        const int k = SL::k_of(s, t, S, v);
        C hv = czero<R>();
        if (v) {
          const double foc = p.f_over_c[k];
          const R fr = FREL ? p.f_rel[k] : R(1);
          double ph = d_los * foc;
          ph -= floor(ph);
          const R a1 = att_los * fr;
          R sn, cs;
          sincos_phase((R)ph, sn, cs);
          hv = mkc(a1 * cs, a1 * sn);
          if constexpr (CH == CH_TWOPATH) {
            double ph2 = d_sec * foc;
            ph2 -= floor(ph2);
            const R a2 = att_sec * fr;
            sincos_phase((R)ph2, sn, cs);
            hv.x -= a2 * cs;
            hv.y -= a2 * sn;
          }
        }
        h[s] = hv;
      }
    }
  }
};

// ---------------------------------------------------------------- the kernel
// Occupancy tuning per instance (trial_inst.hip): MINW = waves/SIMD the register
// allocation targets, NBUF = FFT exchange buffers (2: one barrier per exchange, 1: half
// the LDS), SYMW_LDS = keep the pre-weighted symbols in LDS (thread-private) instead of
// registers.  F = 2048 runs (3, 1, true): 25 KiB LDS and <= 168 VGPRs per 128-thread team.
template <typename R, int F, int T, int NSLOT, bool ALIGNED, int CH, bool CSI, int MINW, int NBUF, bool SYMW_LDS>
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(MINW))) void trial_kernel(TrialParams<R> p0) {
  using C = cx<R>;
  // ---- which point and trial this block runs (uniform binary search over point_start)
  uint32_t pi = 0;
  if (p0.n_points > 1) {
    uint32_t lo = 0, hi = (uint32_t)p0.n_points;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (p0.point_start[mid] <= blockIdx.x) lo = mid; else hi = mid;
    }
    pi = lo;
  }
  using CParams = const __attribute__((address_space(4))) TrialParams<R>;
  CParams& p = *(CParams*)(p0.points + pi);
  constexpr bool WAVEFFT = wave_fft_used(F, T, sizeof(R) == 8);
  // The sub-transforms read their twiddled stages' constants from LDS (stage 1's block and
  // stage 2's rows; fp64: the cot-tan constants of dft8_ct).  CSI instances too, since their
  // per-antenna power table is dynamic LDS sized by A (round 5; before, a static 4 KiB
  // table left no room for stage 2's rows at 3 teams per CU).
  // fp64 up to F 4096: the twiddled stages absorb their twiddles into FMAs (team_fft.h
  // dft8_ct / dft16_ct; F 4096 -1.0 to -1.6 %, CSI -7 to -12 %).  F 8192 keeps the stage
  // twiddles with the prefetched bases: the cot-tan form measured +2.5 % there (its 16-point
  // threads hold the extra constants live across the exchanges; profiles/r05/ab/ab_5su_r05e.json).
  // fp64 F 8192: two 4096-point sub-transforms and a radix-2 stage through lane-half swaps
  // (split_fft.h: two LDS exchanges per transform instead of three)
  constexpr bool SPLITFFT = split_fft_used(F, T, sizeof(R) == 8);
  using FFT = std::conditional_t<
      WAVEFFT, WaveFft<F, T, R, true, true>,
      std::conditional_t<SPLITFFT, SplitFft<F, T, NBUF, R>,
                         TeamFft<F, T, NBUF, R, false, false, false, sizeof(R) == 8 && F <= 4096>>>;
  using SL = Slots<F, T, NSLOT, ALIGNED>;
  // F 4096: the SALU Philox rounds with CSI only -- CSI -2.4 %, perfect CSI +1.1 / +2.0 %
  // (paper / paper CNC 0-8, profiles/r06/k4096/; r03 measured +1.7 % for the perfect-CSI line)
  // F 8192: on since round 6 together with the folded weight (below): config-5 array -1.6 %
  // for both, -1.3 % for the weight alone, +0.4 % for these rounds alone (profiles/r06/k8192/;
  // +1.4 % alone in round 3)
  using CHN = Channel<R, F, T, NSLOT, ALIGNED, CH,
                      (F == 4096 && CSI && MIMO_UNI_4096_CSI != 0) || (F == 8192 && MIMO_UNI_8192 != 0)>;
  constexpr int P = FFT::P;
  constexpr int W = T / 64;
  // Without CSI errors the channel factors as H[a,k] = f_rel[k] H'[a,k]: f_rel cancels in
  // the MRT precoder and in vk_pow, scales r and g by f_rel, and enters only through the
  // AGC power eta and the noise term z = r'/g' + sigma n / (f_rel g').  The antenna loops
  // then run on H' (no per-antenna table reads).  With CSI the estimate's error power
  // mixes sub-carriers, so H keeps the factor.
  constexpr bool FREL = CSI;

  __shared__ C lds[FFT::LDS_TOTAL];
  __shared__ R red[T / 64];  // sized by the team
  __shared__ R vk_part[2][T / 64];
  // alpha formed by one wave per antenna (array_pass): config 2 -1.0 %, CSI -1.2 %, config-5
  // array -2.3 % (profiles/r05/ab/ab_*_alpha1.json).  MIMO_ALPHA1=0: every wave forms it.
  // F 4096 (fp64) since round 6, with the cold paths out of line there: -0.1 % alone, and
  // -1.4 % / -1.0 % together with them (profiles/r06/k4096/; alone +0.8 % in round 5)
  constexpr bool ALPHA1 = MIMO_ALPHA1 != 0 && (F != 4096 || (MIMO_ALPHA1_4096 != 0 && sizeof(R) == 8));
  __shared__ R alpha_s[2];
  // per-antenna mean |H|^2 (CSI model): dynamic LDS of A doubles (the launch sizes it), not
  // a static kMaxCsiAnt table -- the static 4 KiB cost F 4096 its second team per CU and F
  // 2048 its stage-2 twiddle rows (and with them the cot-tan FFT stages)
  extern __shared__ __align__(16) unsigned char dyn_lds[];
  R* pw_csi = reinterpret_cast<R*>(dyn_lds);
  __shared__ C symw_s[SYMW_LDS ? NSLOT * T : 1];  // [slot][thread]
  // wave-split FFT: the one-wave sub-transforms read stage 1's twiddles and (without CSI)
  // stage 2's rows r = 3, 5, 6 from LDS (team_fft.h TWL_N; -24 f64 ops per antenna at config 2)
  constexpr bool LTW1 = WAVEFFT;
  constexpr int TW1_N = [] {
    if constexpr (LTW1) return FFT::TWL_N; else return 1;
  }();
  __shared__ C tw1_s[TW1_N];
  const C* tw1 = LTW1 ? tw1_s : nullptr;

  const int t = threadIdx.x;
  const bool t0 = (t == 0);
  // the thread's sub-carriers: bins tf + T m of the FFT's frequency layout (tf = t except for
  // the split FFT, whose layout is cyclic in a permuted thread index; tf = 0 iff t = 0)
  const int tf = FFT::freq_thread(t);
  const int lane = t & 63, wid = t >> 6;
  const uint32_t trial = (uint32_t)(p.first_trial + (blockIdx.x - p0.point_start[pi]));
  const Key key{(uint32_t)p.seed, (uint32_t)(p.seed >> 32)};
  // CSI error draws: per trial with a rerolled channel (set_precoding_and_recalculate_agc
  // per trial, mp_model.py:206); with a fixed channel (CH_TABLE, reroll_chan=False) the
  // reference draws the erroneous estimate once (Link.__init__, mp_model.py:87) and keeps
  // it for every trial, so all trials share one draw (trial-independent counter).
  const uint32_t csi_trial = CH == CH_TABLE ? kFixedCsiTrial : trial;
  // ... and it belongs to the Link, not to the run: keyed by the engine's csi_seed
  const Key csi_key = CH == CH_TABLE ? Key{(uint32_t)p.csi_seed, (uint32_t)(p.csi_seed >> 32)} : key;
  // Channel counter: the trial, or (diagnostic, chan_period > 0) the trial modulo the
  // period -- every group of chan_period trials replays one sequence of Rayleigh channels,
  // as the reference's forked workers all replay the channel object's seeded generator
  // (channel.py:209-212, mp_model.py:61); bits and noise stay per trial.
  const uint32_t ch_trial = p0.chan_period ? trial % p0.chan_period : trial;
  const int S = p.n_sc, A = p.n_ant, L = p.qam_l, hb = p.half_bits;
  const R inv_sqrt_f = p.inv_sqrt_f;
  if constexpr (sizeof(R) == 8) {  // Box-Muller tables (real.h ln_unit / sincos_lut) into LDS
    for (int i = t; i < kLut64; i += T) lut64[i] = p.lut[i];
  }
  if constexpr (LTW1) {  // the sub-transform's stage-1 block and stage-2 rows (team_fft.h twl_src)
    const C* twsrc = WAVEFFT ? p.tw_wave : p.tw;
    for (int i = t; i < TW1_N; i += T) tw1_s[i] = twsrc[FFT::twl_src(i)];
  }
  if constexpr (sizeof(R) == 8 || LTW1) __syncthreads();

  // RX position for LoS / two-path (mp_model.py:190-201; y uses rx_loc_x, a reference quirk)
  double rx[3] = {0.0, 0.0, 0.0};
  if constexpr (CH == CH_LOS || CH == CH_TWOPATH) {
    const uint4 w = philox4x32_10(make_uint4(0u, trial, ST_LOC, 0u), key);
    const double u0 = (double)w.x * 2.3283064365386963e-10, u1 = (double)w.y * 2.3283064365386963e-10;
    rx[0] = p.rx_x0 - p.rx_var * 0.5 + p.rx_var * u0;
    rx[1] = p.rx_x0 - p.rx_var * 0.5 + p.rx_var * u1;
    rx[2] = p.rx_z;
  }

  // ---- transmitted labels and validity.  Labels are drawn twice (for the symbols before
  // the array pass, for the error counts after it) instead of being held across it.
  uint32_t valid_mask = 0;
  auto gen_labels = [&](int tt, uint32_t (&lab_out)[NSLOT]) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < NSLOT; ++s) {
      bool v;
      const int k = SL::k_of(s, tt, S, v);
      lab_out[s] = v ? qam_label<CHN::kUni>(key, k, trial, p.label_mask) : 0u;
    }
  };
#pragma unroll
  for (int s = 0; s < NSLOT; ++s) {
    bool v;
    SL::k_of(s, tf, S, v);
    valid_mask |= (v ? 1u : 0u) << s;
  }

  // (the thread id laundered per use: the table reads before and after the antenna loop
  // are redone, not kept live across it -- 8 doubles per thread that the F 8192 instance
  // spilled once per trial)
  auto frel_of = [&](int s) __attribute__((always_inline)) -> R {
    if constexpr (FREL) {
      return R(1);
    } else {
      bool v;
      const int k = SL::k_of(s, opaque(tf), S, v);
      return v ? p.f_rel[k] : R(1);
    }
  };

  // ---- pass 1: MRT norms over the (estimated) channel
  R nrm2[NSLOT];
  // CSI: the clean-run combine sum_a H conj(Hhat) / ||Hhat|| (mp_model.py:159-175 with the
  // estimate's precoder) is accumulated here, where H and Hhat are both at hand, and scaled
  // by 1 / ||Hhat|| once pass 1 has the norms -- not in the array pass, where its 16
  // accumulator VGPRs lived across both FFTs (the CSI instance spilled 53 KB per trial of
  // scratch writes, profiles/r05/pmc/pmc_traffic_2csi.json).
  C cc[CSI ? NSLOT : 1];
#pragma unroll
  for (int s = 0; s < NSLOT; ++s) {
    nrm2[s] = R(0);
    if constexpr (CSI) cc[s] = czero<R>();
  }
  const bool clean_cc = CSI && p.incl_clean;
  // pass 1 of the Rayleigh CSI instances in polar form (below; MIMO_CSI_POLAR=0: Cartesian)
  constexpr bool CSI_POLAR = MIMO_CSI_POLAR != 0 && CSI && CH == CH_RAYLEIGH && ALIGNED && sizeof(R) == 8;
  for (int a = 0; a < (MIMO_ABL(p, ABL_PASS1) ? 1 : A); ++a) {
    MIMO_ISA_MARK("pass1");
    const int tl = opaque(tf);
    if constexpr (CH == CH_RAYLEIGH && !CSI) {
      if (!MIMO_ABL(p, ABL_RNG)) {
        R e2[NSLOT];
        CHN::power(p, key, ch_trial, a, tl, e2);
#pragma unroll
        for (int s = 0; s < NSLOT; ++s) nrm2[s] += e2[s];
        continue;
      }
    }
    if constexpr ((CH == CH_LOS || CH == CH_TWOPATH) && !CSI) {
      R e2[NSLOT];
      CHN::power_closed(p, a, tl, rx, e2);
#pragma unroll
      for (int s = 0; s < NSLOT; ++s) nrm2[s] += e2[s];
      continue;
    }
    if constexpr (CSI_POLAR) {
      // Rayleigh + CSI in polar form: with h = rho_h e^{j phi_h} (the FSPL ratio f_c / f_k in
      // rho_h), z = rho_z e^{j phi_z} and Hhat = a h + sc z,
      // |Hhat|^2 = a^2 rho_h^2 + sc^2 rho_z^2 + 2 a sc rho_h rho_z cos(phi_h - phi_z)
      // and h conj(Hhat) = a rho_h^2 + sc rho_h rho_z e^{j (phi_h - phi_z)}: one sine / cosine of
      // the angle words' difference (exact mod 2^32) and one sqrt per slot instead of two full
      // Box-Muller draws and the complex products (mp_model.py:264-282 restated).
      R rh2[NSLOT];
      uint32_t ah[NSLOT];
      const R sa = p.ant_rel[a];
      R pw = R(0);
      CHN::polar(key, ch_trial, ST_CHAN, (uint32_t)a, tl, S, bm_c<R>(sa * sa),
                 [&](int s, R r2, uint32_t w1) __attribute__((always_inline)) {
                   bool v;
                   const R fr = p.f_rel[SL::k_of(s, tl, S, v)];  // H keeps f_c / f_k with CSI (gen<true>)
                   rh2[s] = r2 * (fr * fr);
                   ah[s] = w1;
                   pw += rh2[s];
                 });
      pw = team_sum<T>(pw, red) / (R)S;
      if (t0) pw_csi[a] = pw;
      const R sc = p.csi_b * sqrt_ieee(pw), ca = p.csi_a;
      CHN::polar(csi_key, csi_trial, ST_CSI, (uint32_t)a, tl, S, bm_c<R>(R(1)),
                 [&](int s, R rz2, uint32_t wz) __attribute__((always_inline)) {
                   const R rhz = sqrt_n1(rh2[s] * rz2);  // both > 0: u1 < 1 always
                   R sn, cs;
                   sincos_lut(ah[s] - wz, sn, cs);
                   const R tz = sc * rhz;
                   nrm2[s] = fmar(ca * ca, rh2[s], fmar(sc * sc, rz2, fmar(R(2) * ca * tz, cs, nrm2[s])));
                   if (clean_cc) cc[s] = cadd(cc[s], mkc(fmar(ca, rh2[s], tz * cs), tz * sn));
                 });
      continue;
    }
    C h[NSLOT];
    CHN::template gen<FREL>(p, key, ch_trial, a, tl, rx, h);
    if constexpr (CSI) {
      // mp_model.py:264-282: Hhat = sqrt(1-eps^2) H + eps sqrt(mean_k |H|^2) z
      // (a team_sum -- two barriers -- per antenna: collecting every antenna's wave partials
      // without barriers and regenerating |H|^2 in a pass before this one measured +8 % at
      // config 2 geometry with CSI, profiles/r04/csi/: the barriers cost less than the
      // extra channel draws)
      R pw = R(0);
#pragma unroll
      for (int s = 0; s < NSLOT; ++s) pw = fmar(h[s].x, h[s].x, fmar(h[s].y, h[s].y, pw));
      pw = team_sum<T>(pw, red) / (R)S;
      if (t0) pw_csi[a] = pw;
      C zc[NSLOT];
      CHN::normals(csi_key, csi_trial, ST_CSI, (uint32_t)a, tl, S, zc);
      const R sc = p.csi_b * sqrt_ieee(pw);
      if (clean_cc) {
#pragma unroll
        for (int s = 0; s < NSLOT; ++s) {
          const C e = mkc(fmar(p.csi_a, h[s].x, sc * zc[s].x), fmar(p.csi_a, h[s].y, sc * zc[s].y));
          cc[s] = cadd(cc[s], cmulc(h[s], e));
          h[s] = e;
        }
      } else {
#pragma unroll
        for (int s = 0; s < NSLOT; ++s)
          h[s] = mkc(fmar(p.csi_a, h[s].x, sc * zc[s].x), fmar(p.csi_a, h[s].y, sc * zc[s].y));
      }
    }
#pragma unroll
    for (int s = 0; s < NSLOT; ++s) nrm2[s] = fmar(h[s].x, h[s].x, fmar(h[s].y, h[s].y, nrm2[s]));
  }
  R inv_nrm[NSLOT];
  R etac_p = R(0);  // sum_k ||Hhat_k||^2 for the clean-run noise scaler (mp_model.py:304)
#pragma unroll
  for (int s = 0; s < NSLOT; ++s) {
    const bool v = (valid_mask >> s) & 1u;
    inv_nrm[s] = v ? rsq_r(nrm2[s]) : R(0);
    if constexpr (CSI) cc[s] = cscale(cc[s], inv_nrm[s]);
    const R fr = frel_of(s);
    etac_p += v ? nrm2[s] * (fr * fr) : R(0);
  }
  // etac_p is used only by the clean run after the array pass: pinned here, or the compiler
  // sinks its sum into that conditional block and carries nrm2 and f_rel (16 doubles at
  // F 8192) across the antenna loop -- spilled once per trial
  asm volatile("" : "+v"(etac_p));
  if constexpr (CSI) __syncthreads();  // pw_csi visible

  C d[P];
  C r[NSLOT];
  R g[NSLOT];
#pragma unroll
  for (int s = 0; s < NSLOT; ++s) {
    r[s] = czero<R>();
    g[s] = R(0);
  }

  // ---- array pass: precode -> IFFT -> PA -> FFT -> combine, one antenna at a time.
  // MAIN: symbols = tx labels, combine with the true channel, accumulate g (alpha_a).
  // MCNC: symbols = detected labels, combine with the estimated channel (corrector.py:198-200).
  // The symbols enter pre-weighted, symw = s / ||Hhat|| / sqrt(F) (0 on invalid slots).
  // SYMW_RE (register diet, symbols not in LDS): keep the lattice levels (qam_levels,
  // 1 VGPR per slot) and rebuild the symbol per antenna instead of holding it (4 VGPRs
  // in fp64); the opaque copies stop the compiler from hoisting it back out of the loop.
  // Register diet of the fp64 F = 8192 instance (-2.1 %; at F 2048 the |Hhat|^2 half measured
  // +0.8 %): symbols rebuilt from the labels per antenna, |Hhat|^2 recomputed after the FFT.
  // (every fp64 instance without symbols in LDS: F <= 2048 at 3 waves/SIMD, F 8192)
  constexpr bool SYMW_RE = !SYMW_LDS && sizeof(R) == 8;  // off: +13 % at F 8192
  // Precode with w = 1 / ||Hhat|| / sqrt(F) folded into the channel first (vk then sums
  // |Hhat w|^2 = vk / F): -1.1 % at F 2048 (wave-split instances); +5 % at F 4096, where
  // the 16-point team's register allocation suffers (profiles/r03/ab_o/ab_paper.json).
  // Round 6, with the cold paths out of line: at F 4096 too (not with CSI): paper -2.8 %, paper
  // CNC 0-8 -2.7 % on top of them; paper CSI +3.1 % (profiles/r06/k4096/)
  // ... and at F 8192 (not with CSI): config-5 array -1.3 %, -1.6 % with the SALU Philox rounds
  // (profiles/r06/k8192/ab_5su.json)
  // Not with CSI since round 6: the F 2048 CSI line -1.3 % without it (profiles/r06/k2048/),
  // as at F 4096 (+3.1 % with it)
  constexpr bool PRE_EW = SYMW_RE && ((WAVEFFT && (!CSI || MIMO_PRE_EW_CSI != 0)) ||
                                      (F == 4096 && !CSI && MIMO_PRE_EW_4096 != 0) ||
                                      (F == 8192 && !CSI && MIMO_PRE_EW_8192 != 0));
  // General-p Rapp out of line, and the alpha fallback by the segment table (alpha_fit.h).
  // Rounds 3-5 kept the 16-point F 4096 team's library forms inline (outlined Rapp +1.6 %,
  // r03 ab_s; with the segment table +0.8 %, profiles/r04/alpha/).  Round 6: out of line at F 4096 too -- the instance's scratch 492 -> 288 B/lane, its
  // measured traffic 54 -> 15 KB per trial, paper -1.0 %, paper CSI -1.2 % (profiles/r06/k4096/;
  // +1.6 % in round 3, before the later register cuts)
  constexpr bool COLD_OUT = sizeof(R) == 8 && (F != 4096 || MIMO_COLD_OUT_4096 != 0);
  // |Hhat|^2 for g recomputed after the FFT from the channel (fp64; off: +2.8 % at F 8192,
  // ab_diet_prefetch.json) -- except with CSI, where that would keep the 16-VGPR estimate
  // live across both FFTs next to the true channel: 8 VGPRs of |Hhat|^2 instead.
  constexpr bool E2_RE = sizeof(R) == 8 && !SYMW_LDS && (!CSI || MIMO_E2_RE_CSI != 0);
  C symw_r[SYMW_LDS || SYMW_RE ? 1 : NSLOT];
  // F 8192 (one team per CU, 256 VGPRs): the lattice levels live in LDS ([slot][thread],
  // thread-private: no barrier), not in 8 VGPRs that the allocator reloaded from scratch
  // per antenna.  (Not with CSI: its power table leaves no room.)
  constexpr bool SLAB_LDS = SYMW_RE && F >= 8192 && !CSI && NSLOT * T * 4 <= 16384;
  // In registers at F 4096 (256 VGPRs, 12 scratch reloads per antenna): two slots per word
  // (qam_levels8), -2.2 % on the paper config; at F 2048 (168 VGPRs, no reloads in the loop)
  // one word per slot, the packed form measured neutral to +0.3 % (profiles/r04/levels8/).
  constexpr bool SLAB8 = SYMW_RE && !SLAB_LDS && F == 4096 && MIMO_SLAB8_4096 != 0;
  uint32_t slab_r[SYMW_RE && !SLAB_LDS ? (SLAB8 ? NSLOT / 2 : NSLOT) : 1];
  __shared__ uint32_t slab_s[SLAB_LDS ? NSLOT * T : 1];
  // the lattice point of slot s (the word laundered: rebuilt per antenna, not hoisted)
  auto slab_point = [&](int s) __attribute__((always_inline)) -> C {
    if constexpr (SLAB_LDS) {
      uint32_t l = slab_s[s * T + t];
      asm volatile("" : "+v"(l));
      return levels_point<R>(l);
    } else if constexpr (SLAB8) {
      uint32_t w = slab_r[s >> 1];
      asm volatile("" : "+v"(w));
      return (s & 1) ? levels_point8<R, 1>(w) : levels_point8<R, 0>(w);
    } else {
      uint32_t l = slab_r[s];
      asm volatile("" : "+v"(l));
      return levels_point<R>(l);
    }
  };
  auto set_symbols = [&](const uint32_t (&lab_in)[NSLOT]) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < NSLOT; ++s) {
      if constexpr (SYMW_RE) {
        if constexpr (SLAB_LDS) {
          slab_s[s * T + t] = qam_levels(lab_in[s], L, hb);
        } else if constexpr (SLAB8) {
          const uint32_t v = qam_levels8(lab_in[s], L, hb);
          slab_r[s >> 1] = (s & 1) ? (slab_r[s >> 1] | (v << 16)) : v;
        } else {
          slab_r[s] = qam_levels(lab_in[s], L, hb);
        }
      } else {
        const C v = cscale(qam_point<R>(lab_in[s], L, hb), inv_nrm[s] * inv_sqrt_f);
        if constexpr (SYMW_LDS) symw_s[s * T + t] = v; else symw_r[s] = v;
      }
    }
  };
  auto symw = [&](int s) __attribute__((always_inline)) -> C {
    if constexpr (SYMW_RE) {
      R in = inv_nrm[s];
      asm volatile("" : "+v"(in));
      return cscale(slab_point(s), in * inv_sqrt_f);
    } else if constexpr (SYMW_LDS) {
      return symw_s[s * T + t];
    } else {
      return symw_r[s];
    }
  };
  // WSC: the weight w = 1 / ||Hhat|| / sqrt(F) per slot is what the antenna loops hold
  // (1 / ||Hhat|| is rederived from it after the main pass): no per-antenna multiply and no
  // laundering copy of 1 / ||Hhat||, 8 VALU per antenna: config 2 -0.2 %, MCNC -0.6 %, but the
  // CSI instance +5.3 % (its allocation again), so not with CSI (profiles/r05/ab/ab_*_wsc.json).
  constexpr bool WSC = PRE_EW && !CSI;
  // ... and for the Rayleigh channel the weight is folded into the Box-Muller radius
  // (CHN::normals_w): one multiply per draw instead of three, |h w|^2 from the radius
  constexpr bool WSC_RAY = MIMO_WSC_RAY != 0 && WSC && CH == CH_RAYLEIGH && ALIGNED;  // (fp64: no pipelined draws)
  R wsc[WSC ? NSLOT : 1];
  auto array_pass = [&](bool main_pass, C (&acc)[NSLOT]) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < NSLOT; ++s) acc[s] = czero<R>();
    // Software pipeline (PIPE): antenna a+1's channel draws (one Philox call per chunk)
    // run inside antenna a's FFT exchanges, where the wave otherwise waits on LDS.
    // fp64 at F <= 4096: off (the pipelined draws' registers cost more than the exchange
    // windows hide: -1.8 % without at F 2048, profiles/r02/ab/ab64_2048.json; -2.3 % at
    // F 4096 with the wave-split FFT, scratch 140 -> 36 B/lane, profiles/r02/ab/ab4k_pipe_off.json).
    // fp64 at F 8192: -20 % without (profiles/r02/ab/ab8k_f64_team_pipe.json): fp64 never pipelines.
    constexpr bool PIPE = ALIGNED && CH == CH_RAYLEIGH && !CSI && sizeof(R) == 4;
    C hnext[PIPE ? NSLOT : 1];
    if constexpr (PIPE) {
      const R sa = p.ant_rel[0];
      if (MIMO_ABL(p, ABL_RNG)) CHN::template gen<FREL>(p, key, ch_trial, 0, tf, rx, hnext);
      else CHN::normals(key, ch_trial, ST_CHAN, 0u, tf, S, hnext, bm_c<R>(sa * sa));
    }
    for (int a = 0; a < A; ++a) {
      MIMO_ISA_MARK("array_pass");
      const int tl = opaque(tf);
      C h[NSLOT];
      R rw[WSC_RAY ? NSLOT : 1];  // WSC_RAY: |h w| per slot
      if constexpr (PIPE) {
#pragma unroll
        for (int s = 0; s < NSLOT; ++s) h[s] = hnext[s];
      } else if constexpr (WSC_RAY) {
        if (MIMO_ABL(p, ABL_RNG)) {  // ablation: the synthetic channel, scaled
          CHN::template gen<FREL>(p, key, ch_trial, a, tl, rx, h);
#pragma unroll
          for (int s = 0; s < NSLOT; ++s) {
            h[s] = cscale(h[s], wsc[s]);
            rw[s] = sqrt_ieee(fmar(h[s].x, h[s].x, h[s].y * h[s].y));
          }
        } else {
          const R sa = p.ant_rel[a];
          CHN::normals_w(key, ch_trial, ST_CHAN, (uint32_t)a, tl, S, bm_c<R>(sa * sa), wsc, h, rw);
        }
      } else {
        CHN::template gen<FREL>(p, key, ch_trial, a, tl, rx, h);
        if constexpr (WSC) {
#pragma unroll
          for (int s = 0; s < NSLOT; ++s) h[s] = cscale(h[s], wsc[s]);
        }
      }
      const int an = a + 1 < A ? a + 1 : a;
      const R san = PIPE ? p.ant_rel[an] : R(0);
      // Window w of NW = 2 XCHG exchange windows (IFFT then FFT) draws chunks
      // [w NC / NW, (w + 1) NC / NW) of antenna a+1.  After the last antenna the draws are
      // redone for it and unused: a uniform branch around them measured 2.7 % slower (it
      // splits the exchange windows' basic blocks; profiles/r02/ab/ab32_lastant.json).
      // Ablation ABL_RNG: antenna a+1's synthetic channel, in window 0.
      auto hfill = [&](int w) __attribute__((always_inline)) {
        if constexpr (PIPE) {
          constexpr int NC = CHN::kChunks, NW = 2 * FFT::XCHG;
          if (MIMO_ABL(p, ABL_RNG)) {
            if (w == 0) CHN::template gen<FREL>(p, key, ch_trial, an, tl, rx, hnext);
          } else {
#pragma unroll
            for (int c = 0; c < NC; ++c)
              if (c >= w * NC / NW && c < (w + 1) * NC / NW)
                CHN::normals_chunk(c, key, ch_trial, ST_CHAN, (uint32_t)an, tl, S, hnext, bm_c<R>(san * san));
          }
        }
      };
      auto hfill_ifft = [&](int w) __attribute__((always_inline)) { hfill(w); };
      auto hfill_fft = [&](int w) __attribute__((always_inline)) { hfill(FFT::XCHG + w); };
      C he[CSI ? NSLOT : 1];
      if constexpr (CSI) {
        // (regenerated, not staged: the error term written to HBM in pass 1 and read back
        // here measured +11 %, profiles/r05/ab/ab_2csi_stage_r05e.json)
        C zc[NSLOT];
        CHN::normals(csi_key, csi_trial, ST_CSI, (uint32_t)a, tl, S, zc);
        const R sc = p.csi_b * sqrt_ieee(pw_csi[a]);
#pragma unroll
        for (int s = 0; s < NSLOT; ++s)
          he[s] = mkc(fmar(p.csi_a, h[s].x, sc * zc[s].x), fmar(p.csi_a, h[s].y, sc * zc[s].y));
      }
      auto hest = [&](int s) __attribute__((always_inline)) -> C {
        if constexpr (CSI) return he[s]; else return h[s];
      };
      // vk_part / alpha_s buffer: with ALPHA1 one (the designated wave reads vk_part(a) and
      // every wave alpha(a) before the next antenna's IFFT barrier, which the next writes
      // follow): compile-time LDS addresses; otherwise every wave reads vk_part(a) after the
      // forward FFT, racing the next antenna's writes -- two buffers
      const int vkb = ALPHA1 ? 0 : (a & 1);
      C x[NSLOT];
      R e2[NSLOT];  // |Hhat|^2, kept for g after the FFT
      R vk = R(0);
#pragma unroll
      for (int s = 0; s < NSLOT; ++s) {
        const C e = hest(s);
        if constexpr (PRE_EW) {
          // the lattice point times conj(Hhat w), w = 1 / ||Hhat|| / sqrt(F): vk accumulates
          // |Hhat w|^2 = |Hhat|^2 / ||Hhat||^2 / F directly (11 f64 ops per slot, not 13;
          // vk_scale restores the factor F)
          C ew;
          if constexpr (WSC) {
            ew = e;  // the loops carry h w already
          } else {
            R in = inv_nrm[s];
            asm volatile("" : "+v"(in));
            ew = cscale(e, in * inv_sqrt_f);
          }
          x[s] = cmulc(slab_point(s), ew);
          if constexpr (WSC_RAY) vk = fmar(rw[s], rw[s], vk);
          else vk = fmar(ew.x, ew.x, fmar(ew.y, ew.y, vk));
          if constexpr (!E2_RE) e2[s] = fmar(e.x, e.x, e.y * e.y);
        } else {
          x[s] = cmulc(symw(s), e);  // s conj(Hhat) / ||Hhat|| / sqrt(F); 0 off band (symw = 0)
          e2[s] = fmar(e.x, e.x, e.y * e.y);
          vk = fmar(e2[s], inv_nrm[s] * inv_nrm[s], vk);  // inv_nrm = 0 off band
        }
      }
      if (main_pass) {
        vk = wave_sum_lane63(vk);
        if (lane == 63) vk_part[vkb][wid] = vk;  // read after the IFFT's first barrier
      }
      SL::scatter(d, x, t0);
      // the FFTs take the thread id already laundered for this antenna (tl) where it is the
      // physical one: their own opaque copy of it then costs no register move in run_second
      const int tfft = SPLITFFT ? t : tl;
      if (!MIMO_ABL(p, ABL_FFT))
        FFT::template run<+1, 0, SL::zero_mask()>(d, lds, WAVEFFT ? p.tw_wave : p.tw, tfft, MIMO_ABL(p, ABL_XCHG), hfill_ifft,
                                                  tw1);
      if (!MIMO_ABL(p, ABL_PA)) pa_block<COLD_OUT>(p.pa_kind, d, p.sat_tx, p.sqrt_sat_tx, p.inv_sat_tx, p.rapp_p, p.toi_tx);
      // alpha_a (Bussgang gain of antenna a's PA from its precoding power, main pass only)
      auto alpha_of_vk = [&]() __attribute__((always_inline)) -> R {
        R vks = vk_part[vkb][0];
#pragma unroll
        for (int i = 1; i < W; ++i) vks += vk_part[vkb][i];
        const R x = fmar(vks, PRE_EW ? p.inv_vk0_f : p.inv_vk0, -R(1));
        // Polynomial alpha: -7 % at F = 2048, but +3 % at F = 8192 (SGPR pressure of the
        // 8 waves/team instance, tools/ab_libs.py), so only up to F = 4096.
        if (sizeof(R) == 4 && F <= 4096 && absr(x) <= p.alpha_xlim) {
          R acc = p.apoly[8];
#pragma unroll
          for (int i = 7; i >= 0; --i) acc = fmar(acc, x, p.apoly[i]);
          return acc;
        } else if (sizeof(R) == 8 && absr(x) <= p.alpha_xlim) {
          // Horner, 18 FMAs with the coefficients as SGPR operands instead of the library
          // exp + erfc.  (Plain fma() compiles to v_fmac_f64 and copies every coefficient
          // into the accumulator's VGPRs first, 2 v_mov per step: +0.7 % at F 2048, +0.9 %
          // at F 4096, profiles/r03/ab_o.)
          double acc = p.amono64[18];
#pragma unroll
          for (int k = 17; k >= 0; --k) {
            const double ck = p.amono64[k];
            asm("v_fma_f64 %0, %1, %2, %3" : "=v"(acc) : "v"(acc), "v"((double)x), "s"(ck));
          }
          return (R)acc;
        } else {
          // (the register-diet pass sums vk / F: vks F is the precoding power)
          const R g2 = p.alpha_c / (PRE_EW ? vks * (R)F : vks);
          // fp64: the segment table (alpha_fit.h, appended to the Box-Muller tables in HBM)
          if constexpr (COLD_OUT) return alpha_seg(g2, reinterpret_cast<const double*>(p.lut + kLut64));
          else return alpha_of_gamma2(g2);
        }
      };
      // ALPHA1: one wave per antenna (a mod W) forms it from the vk partials (visible since the
      // IFFT's first barrier) and hands it over in LDS; the forward FFT's cross-wave barrier
      // orders the hand-off (alpha_s double-buffered like vk_part).  The other waves skip the
      // partial sum and the 18-FMA polynomial.
      if constexpr (ALPHA1) {
        // (ablation builds without the transforms' barriers: order the vk_part hand-off)
        if (MIMO_ABL(p, ABL_FFT) || MIMO_ABL(p, ABL_XCHG)) __syncthreads();
        if (main_pass && wid == (a & (W - 1))) {
          const R al = alpha_of_vk();
          if (lane == 0) alpha_s[vkb] = al;
        }
      }
      if (!MIMO_ABL(p, ABL_FFT))
        FFT::template run_second<-1>(d, lds, WAVEFFT ? p.tw_wave : p.tw, tfft, MIMO_ABL(p, ABL_XCHG), hfill_fft, tw1);
      if constexpr (PIPE) {
        if (MIMO_ABL(p, ABL_FFT)) {  // no transforms ran, so no exchange windows (ABL_XCHG keeps them)
#pragma unroll
          for (int w = 0; w < 2 * FFT::XCHG; ++w) hfill(w);
        }
      }
      // keep the vk_part / alpha_s hand-offs ordered when the ablations drop the barriers
      if (MIMO_ABL(p, ABL_FFT) || (ALPHA1 && MIMO_ABL(p, ABL_XCHG))) __syncthreads();
      R alpha_a = R(0);
      if (main_pass) alpha_a = ALPHA1 ? alpha_s[vkb] : alpha_of_vk();
#pragma unroll
      for (int s = 0; s < NSLOT; ++s) {
        const C y = SL::gather(d, s, t0);
        if (main_pass) {
          acc[s] = cmac(acc[s], h[s], y);
          if constexpr (E2_RE) {
            C e = hest(s);
            asm volatile("" : "+v"(e.x), "+v"(e.y));
            g[s] = fmar(alpha_a, fmar(e.x, e.x, e.y * e.y), g[s]);
          } else {
            g[s] = fmar(alpha_a, e2[s], g[s]);  // sum_a alpha_a |Hhat|^2; x 1/||Hhat|| after the pass
          }
        } else {
          acc[s] = cmac(acc[s], hest(s), y);
        }
      }
    }
#pragma unroll
    for (int s = 0; s < NSLOT; ++s) {
      // WSC: sum_a (h w) y = w sum_a h y
      if constexpr (WSC) acc[s] = cscale(acc[s], wsc[s] > R(0) ? inv_sqrt_f / wsc[s] : R(0));
      else acc[s] = cscale(acc[s], inv_sqrt_f);
    }
  };

  {
    uint32_t lab0[NSLOT];
    gen_labels(tf, lab0);
    set_symbols(lab0);
  }
  if constexpr (WSC) {
#pragma unroll
    for (int s = 0; s < NSLOT; ++s) wsc[s] = inv_nrm[s] * inv_sqrt_f;
  }
  array_pass(true, r);
  if constexpr (WSC) {
#pragma unroll
    for (int s = 0; s < NSLOT; ++s) inv_nrm[s] = wsc[s] / inv_sqrt_f;
  }
#pragma unroll
  for (int s = 0; s < NSLOT; ++s) {
    // WSC: g accumulated alpha |h w|^2 = w^2 alpha |h|^2, and inv_nrm / w^2 = 1 / (w / sqrt(F))
    if constexpr (WSC) g[s] = wsc[s] > R(0) ? g[s] / (wsc[s] * inv_sqrt_f) : R(0);
    else g[s] *= inv_nrm[s];
  }
  uint32_t lab[NSLOT];
  gen_labels(opaque(tf), lab);

  // ---- AWGN + AGC (noise.py:56-83 on all bins; only in-band bins matter)
  C zn[NSLOT];
  CHN::normals(key, trial, ST_NOISE, 0u, tf, S, zn);
  R eta_p = R(0);
#pragma unroll
  for (int s = 0; s < NSLOT; ++s) {
    const R gs = g[s] * frel_of(s);
    eta_p = ((valid_mask >> s) & 1u) ? fmar(gs, gs, eta_p) : eta_p;
  }
  const R eta = team_sum<T>(eta_p, red) / (R)S;
  uint32_t* out = p0.counts + (size_t)blockIdx.x * p0.n_idx;

  auto record = [&](int idx, uint32_t errs) __attribute__((always_inline)) {
    const R tot = team_sum<T>((R)errs, red);
    if (t0) out[idx] = (uint32_t)(tot + R(0.5));
  };

  if (p.incl_clean) {
    // clean run (mp_model.py:159-175): no PA, AGC / noise from sum_a Hhat P = ||Hhat||
    const R etac = team_sum<T>(etac_p, red) / (R)S;
    const R sig_c = sqrt_ieee(p.es_over_snr * etac);
    uint32_t errs = 0;
#pragma unroll
    for (int s = 0; s < NSLOT; ++s) {
      const C sym = qam_point<R>(lab[s], L, hb);
      C rc;
      if constexpr (CSI) rc = cmul(cc[s], sym); else rc = cscale(sym, inv_nrm[s] > R(0) ? R(1) / inv_nrm[s] : R(0));
      const R ig = inv_nrm[s];  // 1 / ||Hhat||  (/ f_rel when factored)
      const R sn = sig_c / frel_of(s);
      const C zc = mkc((rc.x + sn * zn[s].x) * ig, (rc.y + sn * zn[s].y) * ig);
      const uint32_t lh = slice(zc, L, hb);
      errs += ((valid_mask >> s) & 1u) ? __popc(lh ^ lab[s]) : 0u;
    }
    record(0, errs);
  }

  const R sig = sqrt_ieee(p.es_over_snr * eta);
  C z[NSLOT];
#pragma unroll
  for (int s = 0; s < NSLOT; ++s) {
    const R ig = ((valid_mask >> s) & 1u) ? R(1) / g[s] : R(0);
    const R sn = sig / frel_of(s);
    z[s] = mkc((r[s].x + sn * zn[s].x) * ig, (r[s].y + sn * zn[s].y) * ig);
  }

  // ---- CNC / MCNC receiver.  One loop per receiver kind (a uniform branch outside the
  // loops): the CNC loop then holds neither the MCNC-only state (g, 1/||Hhat||, the
  // symbols' LDS) nor its code, so it runs without the register spills a shared loop had.
  C dist[NSLOT];
#pragma unroll
  for (int s = 0; s < NSLOT; ++s) dist[s] = czero<R>();
  int idx = p.incl_clean;
  // slice z - dist, count and record iteration `it`; false once the last one is recorded
  auto detect = [&](int it, uint32_t (&lh)[NSLOT]) __attribute__((always_inline)) -> bool {
    uint32_t errs = 0;
#pragma unroll
    for (int s = 0; s < NSLOT; ++s) {
      lh[s] = slice(csub(z[s], dist[s]), L, hb);
      errs += ((valid_mask >> s) & 1u) ? __popc(lh[s] ^ lab[s]) : 0u;
    }
    if ((p.rec_mask >> it) & 1u) record(idx++, errs);
    return it < p.max_iter;
  };
  if (p.receiver == RX_CNC) {
    for (int it = 0;; ++it) {
      uint32_t lh[NSLOT];
      if (!detect(it, lh)) break;
      // corrector.py:84-110: single-antenna re-synthesis of the clipping distortion
      C x[NSLOT];
#pragma unroll
      for (int s = 0; s < NSLOT; ++s)
        x[s] = ((valid_mask >> s) & 1u) ? cscale(qam_point<R>(lh[s], L, hb), inv_sqrt_f) : czero<R>();
      SL::scatter(d, x, t0);
      FFT::template run<+1, 0, SL::zero_mask()>(d, lds, WAVEFFT ? p.tw_wave : p.tw, t, false,
                                                typename FFT::NoFill{}, tw1);
      pa_block<COLD_OUT>(p.cnc_pa_kind, d, p.sat_cnc, p.sqrt_sat_cnc, p.inv_sat_cnc, p.rapp_p, p.toi_cnc);
      FFT::template run_second<-1>(d, lds, WAVEFFT ? p.tw_wave : p.tw, t, false, typename FFT::NoFill{}, tw1);
      const R sc = inv_sqrt_f * p.inv_alpha_cnc;
#pragma unroll
      for (int s = 0; s < NSLOT; ++s) {
        const C y = SL::gather(d, s, t0);
        dist[s] = ((valid_mask >> s) & 1u) ? csub(cscale(y, sc), qam_point<R>(lh[s], L, hb)) : czero<R>();
      }
    }
  } else {
    // corrector.py:165-207: re-transmit the detected symbols through the whole array
    for (int it = 0;; ++it) {
      uint32_t lh[NSLOT];
      if (!detect(it, lh)) break;
      C est[NSLOT];
      set_symbols(lh);
      array_pass(false, est);
#pragma unroll
      for (int s = 0; s < NSLOT; ++s) {
        const R ig = ((valid_mask >> s) & 1u) ? R(1) / g[s] : R(0);
        dist[s] = ((valid_mask >> s) & 1u) ? csub(cscale(est[s], ig), qam_point<R>(lh[s], L, hb))
                                           : czero<R>();
      }
    }
  }
}

}  // namespace mimo
