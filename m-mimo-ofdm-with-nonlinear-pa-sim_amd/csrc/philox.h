// Device-side Philox4x32-10 and the engine's random-stream layout (gfx950).
//
// One statement of the layout lives in oracle/philox.py (the CPU checker); this is the
// device statement, and tests/test_gpu_*.py pin the two against each other.
//   key = (seed_lo32, seed_hi32);  counter = (element, trial, stream, aux)
//   BITS  (k>>2, trial, 1, 0)  -> word[k&3] & (M-1) = QAM label of sub-carrier k
//   CHAN  (q,    trial, 2, a)  -> 2 CN(0,1) draws, sub-carrier pair q, antenna a
//   NOISE (q,    trial, 3, 0)  -> 2 CN(0,1) draws
//   CSI   (q,    trial, 4, a)  -> 2 CN(0,1) draws
//   LOC   (0,    trial, 5, 0)  -> 2 uniforms (RX position jitter)
// Replaces the reference's sequential PCG64 streams (mp_model.py:121-125,
// channel.py:209-212) with counter-addressed ones so that every trial is reproducible
// on any device count and in any order.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "real.h"

namespace mimo {

enum Stream : uint32_t { ST_BITS = 1, ST_CHAN = 2, ST_NOISE = 3, ST_CSI = 4, ST_LOC = 5 };

struct Key {
  uint32_t k0, k1;
};

// a ^ b ^ k in one VALU op: gfx950 has no v_xor3_b32 but has v_bitop3_b32 (LUT 0x96).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t k) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(k));
  return r;
}

// One round = 2 x v_mad_u64_u32 (the full 64-bit product in one ~4-cycle wave64
// instruction) + 2 x v_bitop3_b32, instead of mul_hi + mul_lo + 2 xor per word: every
// 32-bit integer op is half rate on gfx950 (tools/microbench/ops.hip).  The key words are
// uniform (SGPRs), the one scalar operand a VOP3 op may take.

// UNI = true: every call site's counter words 1-3 (trial, stream, antenna) are
// wave-uniform, so rounds 0-2 are written in plain C where a uniform operand meets the
// round: the compiler keeps those products and xors on the SALU (round 0: M1 c.z; round 1:
// M0 c.x) and needs one v_xor where bitop3 would first copy the uniform word into a VGPR;
// rounds 3-9 are per-lane throughout.  Measured: -1.2 % at F 2048 and -4 % on the CSI
// instance, but +1.7 % / +1.4 % at F 4096 / 8192 (profiles/r03/ab_o, ab_p), so the
// trial kernel takes it for the fp64 wave-split instances only (Channel::kUni).
template <bool UNI = false>
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, Key key) {
  if constexpr (!UNI) {
    uint32_t k0 = key.k0, k1 = key.k1;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      if (r) {
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
      }
      const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
      const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
      c = make_uint4(xor3((uint32_t)(p1 >> 32), c.y, k0), (uint32_t)p1, xor3((uint32_t)(p0 >> 32), c.w, k1),
                     (uint32_t)p0);
    }
    return c;
  } else {
    constexpr uint32_t kW0 = 0x9E3779B9u, kW1 = 0xBB67AE85u;
    const uint32_t k0 = key.k0, k1 = key.k1;
    // round 0: c.y, c.z, c.w uniform (readfirstlane keeps c.w ^ k1 one SGPR operand; the
    // compiler would otherwise re-associate it into two v_xor)
    uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t wk = (uint32_t)__builtin_amdgcn_readfirstlane((int)(c.w ^ k1));
    c = make_uint4((uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ wk, (uint32_t)p0);
    // round 1: c.x, c.y uniform
    p0 = (uint64_t)0xD2511F53u * c.x;
    p1 = (uint64_t)0xCD9E8D57u * c.z;
    c = make_uint4((uint32_t)(p1 >> 32) ^ (c.y ^ (k0 + kW0)), (uint32_t)p1, ((uint32_t)(p0 >> 32) ^ (k1 + kW1)) ^ c.w,
                   (uint32_t)p0);
    // round 2: c.w uniform
    p0 = (uint64_t)0xD2511F53u * c.x;
    p1 = (uint64_t)0xCD9E8D57u * c.z;
    c = make_uint4(xor3((uint32_t)(p1 >> 32), c.y, k0 + 2u * kW0), (uint32_t)p1,
                   (uint32_t)(p0 >> 32) ^ (c.w ^ (k1 + 2u * kW1)), (uint32_t)p0);
#pragma unroll
    for (int r = 3; r < 10; ++r) {
      p0 = (uint64_t)0xD2511F53u * c.x;
      p1 = (uint64_t)0xCD9E8D57u * c.z;
      c = make_uint4(xor3((uint32_t)(p1 >> 32), c.y, k0 + (uint32_t)r * kW0), (uint32_t)p1,
                     xor3((uint32_t)(p0 >> 32), c.w, k1 + (uint32_t)r * kW1), (uint32_t)p0);
    }
    return c;
  }
}

// Box-Muller on two words -> CN(0,1):  sqrt(-ln u1) * exp(j 2 pi u2),
// u1 = (w0 + 0.5) 2^-32, u2 = w1 2^-32 (oracle/philox.py box_muller).
//
// fp32: v_sin/v_cos take revolutions, so 2*pi*u2 is never formed; v_log is log2, and the
// scale argument c = -ln(2) scale^2 returns scale * CN(0,1) at no extra cost.
// fp64: LDS-table ln / sincos and a Newton sqrt (real.h, ~1.5 ulp); c = -scale^2 (natural log).
// bm_c<R>(scale^2) builds c for either.
constexpr float kNegLn2 = -0.69314718055994531f;
template <typename R>
__device__ __forceinline__ R bm_c(R scale2);
template <>
__device__ __forceinline__ float bm_c<float>(float scale2) {
  return kNegLn2 * scale2;
}
template <>
__device__ __forceinline__ double bm_c<double>(double scale2) {
  return -scale2;
}

__device__ __forceinline__ float bm_log(uint32_t w0, float) {
  return __builtin_amdgcn_logf(fmaf((float)w0, 2.3283064365386963e-10f, 1.1641532182693481e-10f));
}
// fp64: LDS-table ln (real.h ln_unit; the trial kernel loads lut64 first).  The series
// forms (ln_pos, sincos_rev) measured 1.4-3.9 % slower.
__device__ __forceinline__ double bm_log(uint32_t w0, double) {
  // ln of u1 = (w0 + 0.5) 2^-32 from the bits of w0 + 0.5 (exact) with the 2^-32 taken into
  // ln_unit's exponent: no scaling instruction
  return ln_unit<-32>((double)w0 + 0.5);
}

__device__ __forceinline__ float2 box_muller(uint32_t w0, uint32_t w1, float c = kNegLn2) {
  const float u1 = fmaf((float)w0, 2.3283064365386963e-10f, 1.1641532182693481e-10f);
  const float u2 = (float)w1 * 2.3283064365386963e-10f;
  // Raw v_sqrt_f32 (1 ulp): __builtin_sqrtf expands to ~15 instructions of IEEE
  // correction.  u2 may round up to 1.0 (w1 > 2^32 - 128), which v_sin/v_cos treat as
  // one full revolution, i.e. as 0.
  const float rho = __builtin_amdgcn_sqrtf(c * __builtin_amdgcn_logf(u1));
  return make_float2(rho * __builtin_amdgcn_cosf(u2), rho * __builtin_amdgcn_sinf(u2));
}
__device__ __forceinline__ double2 box_muller(uint32_t w0, uint32_t w1, double c) {
  const double rho = sqrt_n1(c * bm_log(w0, 0.0));  // argument > 0: u1 < 1 always
  double s, co;
  sincos_lut(w1, s, co);  // revolutions w1 2^-32, from the word itself
  return make_double2(rho * co, rho * s);
}

// sw: return the two draws swapped (z1 from words z, w); the swap selects the 32-bit words,
// not the finished complex values (4 selects instead of 8 in float64).
template <bool UNI = false, class C>
__device__ __forceinline__ void cn_pair(Key key, uint32_t q, uint32_t trial, uint32_t stream, uint32_t aux, C& z1,
                                        C& z2, real_of<C> c, bool sw = false) {
  const uint4 w = philox4x32_10<UNI>(make_uint4(q, trial, stream, aux), key);
  z1 = box_muller(sw ? w.z : w.x, sw ? w.w : w.y, c);
  z2 = box_muller(sw ? w.x : w.z, sw ? w.y : w.w, c);
}

// |z1|^2, |z2|^2 of cn_pair's draws without forming them: rho^2 = c log(u1) (one log
// per draw; no sqrt / sin / cos).  MRT norms only need the channel power.
template <bool UNI = false, typename R>
__device__ __forceinline__ void cn_pair_pow(Key key, uint32_t q, uint32_t trial, uint32_t stream, uint32_t aux, R& p1,
                                            R& p2, R c, bool sw = false) {
  const uint4 w = philox4x32_10<UNI>(make_uint4(q, trial, stream, aux), key);
  p1 = c * bm_log(sw ? w.z : w.x, R(0));
  p2 = c * bm_log(sw ? w.x : w.z, R(0));
}

// Quarter pairing: sub-carrier k -> pair index q and slot (0: k1, 1: k2 = k1 + S/4).
__device__ __forceinline__ void pair_of(int k, int n_sc, uint32_t& q, int& slot) {
  const int half = n_sc >> 1, quarter = n_sc >> 2;
  const int h = k >= half ? 1 : 0;
  const int r = k - h * half;
  slot = r >= quarter ? 1 : 0;
  q = (uint32_t)(h * quarter + r - slot * quarter);
}

template <bool UNI = false>
__device__ __forceinline__ uint32_t qam_label(Key key, int k, uint32_t trial, uint32_t mask) {
  const uint4 w = philox4x32_10<UNI>(make_uint4((uint32_t)k >> 2, trial, ST_BITS, 0u), key);
  const int s = k & 3;
  const uint32_t word = s == 0 ? w.x : s == 1 ? w.y : s == 2 ? w.z : w.w;
  return word & mask;
}

}  // namespace mimo
