// libmimo_engine: C-ABI host side of the MI355X Monte-Carlo BER engine.
//
// Coarse seam = mp_model.Link (mp_model.py:32-329).  mimo_engine_run launches the fused
// trial kernel (trial_kernel.h) over a batch of trials, reduces the per-trial counts on
// the device and adds the totals into the caller's counters, like Link.simulate adds
// into its shared mp.Array counters (mp_model.py:217-222).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/mimo_engine.h"
#include "trial_launch.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                          \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess) return fail(MIMO_EHIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

constexpr double kSpeedOfLight = 299792458.0;  // scipy.constants.c

bool is_pow2(long v) { return v > 0 && (v & (v - 1)) == 0; }

// Per-point sums of the per-trial counts of one launch: block (k, idx) adds the counts of
// trial blocks [first[k], first[k + 1]) -- a slice of at most kSlice trials of one point --
// into tot[point_of[k]][idx] (integer sums: the order does not matter; one 64-bit atomic
// per wave).
constexpr uint32_t kSlice = 4096;
__global__ void reduce_counts(const uint32_t* __restrict__ c, const uint32_t* __restrict__ first,
                              const int32_t* __restrict__ point_of, int n_idx, unsigned long long* __restrict__ tot) {
  const int k = blockIdx.x, idx = blockIdx.y;
  unsigned long long acc = 0;
  for (uint32_t t = first[k] + threadIdx.x; t < first[k + 1]; t += blockDim.x) acc += c[(size_t)t * n_idx + idx];
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(&tot[(size_t)point_of[k] * n_idx + idx], acc);
}

// Bussgang gain of modulation.py:178-189 as a function of gamma^2.
double alpha_exact(double g2) {
  const double g = std::sqrt(g2);
  return 1.0 - std::exp(-g2) + 0.88622692545275801 * g * std::erfc(g);
}

// Degree-8 fit of alpha(g0^2 / (1 + x)) on |x| <= 0.25 (x = relative deviation of an
// antenna's precoding power from its mean S/A, a few % for MRT): Chebyshev interpolation
// at 64 nodes, converted to monomials in x for a Horner evaluation in fp32.  Max relative
// error ~1e-7 for IBO in [-10, 30] dB (fp32 rounding level); the kernel falls back to
// the exact formula outside the interval.
struct AlphaFit {
  double apoly[9];   // fp32 Horner monomials in x
  double xlim;
  double amono[19];  // fp64 Horner monomials in x (degree 18)
};

AlphaFit fit_alpha(double g0sq) {
  AlphaFit p{};
  constexpr int N = 64, D = 8;
  constexpr double L = 0.25;
  double c[D + 1] = {0};
  for (int j = 0; j < N; ++j) {
    const double th = M_PI * (j + 0.5) / N, t = std::cos(th);
    const double f = alpha_exact(g0sq / (1.0 + L * t));
    for (int k = 0; k <= D; ++k) c[k] += f * std::cos(k * th) * (k == 0 ? 1.0 : 2.0) / N;
  }
  // Chebyshev -> monomials in t (T_{k+1} = 2 t T_k - T_{k-1}), then t = x / L
  double Tm1[D + 1] = {0}, T0[D + 1] = {0}, mono[D + 1] = {0};
  T0[0] = 1.0;
  for (int k = 0; k <= D; ++k) {
    for (int i = 0; i <= D; ++i) mono[i] += c[k] * T0[i];
    double Tn[D + 1] = {0};
    for (int i = 0; i <= D; ++i) {
      if (i > 0) Tn[i] += (k == 0 ? 1.0 : 2.0) * T0[i - 1];  // T_1 = t
      Tn[i] -= Tm1[i];
    }
    for (int i = 0; i <= D; ++i) {
      Tm1[i] = T0[i];
      T0[i] = Tn[i];
    }
  }
  double sc = 1.0;
  for (int i = 0; i <= D; ++i, sc /= L) p.apoly[i] = mono[i] * sc;
  p.xlim = L;
  // fp64: Chebyshev interpolant of degree 18 on the same interval at 64 nodes, in long
  // double, converted to monomials in x (Horner in the kernel: 18 FMAs with the
  // coefficients in SGPRs, instead of Clenshaw's 36 ops).  The Taylor radius is 4
  // half-widths (the pole of g0^2 / (1 + x) at x = -1), so the monomials stay O(1) and
  // the Horner sum is as accurate as Clenshaw: <= 1.6e-16 relative against the long
  // double formula over 2e6 points for IBO -5 ... 30 dB (the Clenshaw form: <= 2.1e-16).
  constexpr int D64 = 18;
  long double ck[D64 + 1];
  for (int k = 0; k <= D64; ++k) {
    long double s = 0.0L;
    for (int j = 0; j < N; ++j) {
      const long double th = 3.14159265358979323846264338327950288L * (j + 0.5L) / N;
      const long double t = std::cos(th);
      const long double g2 = (long double)g0sq / (1.0L + (long double)L * t);
      const long double g = std::sqrt(g2);
      const long double f = 1.0L - std::exp(-g2) + 0.886226925452758013649083741671L * g * std::erfc(g);
      s += f * std::cos(k * th);
    }
    ck[k] = s * (k == 0 ? 1.0L : 2.0L) / N;
  }
  long double Um1[D64 + 1] = {0}, U0[D64 + 1] = {0}, um[D64 + 1] = {0};
  U0[0] = 1.0L;
  for (int k = 0; k <= D64; ++k) {
    for (int i = 0; i <= D64; ++i) um[i] += ck[k] * U0[i];
    long double Un[D64 + 1] = {0};
    for (int i = 0; i <= D64; ++i) {
      if (i > 0) Un[i] += (k == 0 ? 1.0L : 2.0L) * U0[i - 1];
      Un[i] -= Um1[i];
    }
    for (int i = 0; i <= D64; ++i) {
      Um1[i] = U0[i];
      U0[i] = Un[i];
    }
  }
  long double scl = 1.0L;
  for (int i = 0; i <= D64; ++i, scl /= (long double)L) p.amono[i] = (double)(um[i] * scl);
  return p;
}

// fp64 Box-Muller tables (real.h ln_unit / sincos_lut), computed in long double, followed
// by the Bussgang-gain segment table (alpha_fit.h; stays in HBM, the kernel copies only the
// first kLut64 entries into LDS).
constexpr int kLut64Alloc = mimo::kLut64 + (mimo::kAlphaTabDoubles + 1) / 2;
std::vector<double2> lut64_table() {
  std::vector<double2> t(kLut64Alloc);
  {
    const std::vector<double> at = mimo::alpha_segment_table();
    double* dst = reinterpret_cast<double*>(t.data() + mimo::kLut64);
    for (int i = 0; i < mimo::kAlphaTabDoubles; ++i) dst[i] = at[i];
  }
  {  // real.h ln_unit: bucket i = m in [0.5 + i 2^-10, 0.5 + (i + 1) 2^-10), c = 1 for the top one
    for (int i = 0; i < mimo::kLnTab; ++i) {
      double c = 1.0;
      if (i != mimo::kLnTab - 1) {
        const long double ctr = 0.5L + (i + 0.5L) / 1024.0L;
        int ex;
        const long double fr = std::frexp(1.0L / ctr, &ex);
        c = (double)std::ldexp(std::round(std::ldexp(fr, 12)), ex - 12);
      }
      t[i] = make_double2(c, (double)(-std::log((long double)c)));
    }
  }
  for (int i = 0; i < mimo::kScTab; ++i) {
    const long double a = 2.0L * 3.14159265358979323846264338327950288L * i / mimo::kScTab;
    t[mimo::kLnTab + i] = make_double2((double)std::cos(a), (double)std::sin(a));
  }
  return t;
}

}  // namespace

namespace mimo {
void set_error(const std::string& m) { g_err = m; }
}  // namespace mimo

struct mimo_engine {
  mimo_config cfg{};
  std::vector<double> tx_pos, freqs;
  std::vector<double> chan_inband;        // MIMO_CH_TABLE: [A][S] (re, im), sub-carrier order k
  mimo_point pt{};
  bool have_point = false;
  // device state (created lazily on the first run: fork safety)
  bool ready = false;
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  float2* d_tw[2] = {nullptr, nullptr};  // fp32 stage twiddles for team_size(F), alt_team_size(F)
  double2* d_tw64 = nullptr;              // fp64 stage twiddles for team_size64(F)
  double2* d_twave64 = nullptr;           // wave-split FFT twiddles (wave_fft.h) where the instance uses it
  float2* d_twave32 = nullptr;
  double2* d_lut64 = nullptr;             // fp64 Box-Muller tables (lut64_table)
  float2* d_tab32 = nullptr;              // MIMO_CH_TABLE channel, fp32 / fp64 copies
  double2* d_tab64 = nullptr;
  float* d_ant_rel = nullptr;
  float* d_f_rel = nullptr;
  double* d_ant_rel64 = nullptr;
  double* d_f_rel64 = nullptr;
  double* d_f_over_c = nullptr;
  double* d_tx_pos = nullptr;
  uint32_t* d_counts = nullptr;
  size_t counts_cap = 0;
  unsigned long long* d_tot = nullptr;    // [points][n_idx] totals of one run
  size_t tot_cap = 0;
  // per-launch tables in one device blob, filled by one copy from a pinned host buffer:
  // TrialParams<R>[segments] | uint32 block offsets [segments + 1] |
  // uint32 reduction-slice starts [slices + 1] (<= kSlice trials, one point each) | int32 point of slice [slices]
  char* d_blob = nullptr;
  char* h_blob = nullptr;
  size_t blob_cap = 0, hblob_cap = 0;
  double d0 = 1.0;
  double last_ms = 0.0;
  // fit_alpha results per IBO (bit pattern of 10^(IBO/10)): the long-double fit costs
  // ~0.3 ms, paid once per IBO instead of once per point and batch of a sweep
  std::unordered_map<uint64_t, AlphaFit> alpha_fits;
  std::string desc;
};

namespace {

int team_for(int F) { return mimo::team_size(F); }

mimo::InstanceKey select_instance(const mimo_engine* e, bool csi) {
  mimo::InstanceKey k{};
  k.F = e->cfg.n_fft;
  k.f64 = e->cfg.precision != MIMO_PREC_F32;
  const int S = e->cfg.n_sub_carr;
  auto aligned_at = [&](int T) {
    const int P = k.F / T;
    return (S % (4 * T) == 0) && S < k.F && (S / T == 8 || S / T == 4) && (S / T) < P;
  };
  k.T = k.f64 ? mimo::team_size64(k.F) : team_for(k.F);
  if (k.f64) {  // one team size per fp64 instance
    const int P = k.F / k.T;
    k.aligned = aligned_at(k.T);
    k.nslot = k.aligned ? S / k.T : P;
    k.ch = e->cfg.channel_kind;
    k.csi = csi;
    return k;
  }
  // Unaligned bands (S % 4T != 0) run the generic predicated path with P slots per
  // thread; the alternative team has half the points per thread, which measured 1.5x
  // faster there (60.7 vs 40.7 ms at S = 1000, F = 2048; profiles/r01/ab_generic.json).
  if (!aligned_at(k.T) && mimo::alt_team_size(k.F) != k.T) k.T = mimo::alt_team_size(k.F);
  if (const char* env = std::getenv("MIMO_TEAM")) {  // A/B override: MIMO_TEAM=<threads per trial>
    const int t = std::atoi(env);
    if (t == mimo::alt_team_size(k.F) || t == mimo::team_size(k.F)) k.T = t;
  }
  const int P = k.F / k.T;
  k.aligned = aligned_at(k.T);
  k.nslot = k.aligned ? S / k.T : P;
  k.ch = e->cfg.channel_kind;
  k.csi = csi;
  return k;
}

template <typename R>
hipError_t launch(const mimo::InstanceKey& k, dim3 grid, hipStream_t st, const mimo::TrialParams<R>& p, bool* found,
                  hipFuncAttributes* attr = nullptr) {
  constexpr bool F64 = sizeof(R) == 8;
#define MIMO_LAUNCH_F(FV)                                                                    \
  if constexpr (F64) return mimo::launch_trial_F##FV##_f64(k, grid, st, p, found, attr);     \
  else return mimo::launch_trial_F##FV##_f32(k, grid, st, p, found, attr);
#ifdef MIMO_ONLY_F  // single-size diagnostic / A-B builds (Makefile targets ablation, variant)
  if (k.F == MIMO_ONLY_F) {
#if MIMO_ONLY_F == 2048
    MIMO_LAUNCH_F(2048)
#elif MIMO_ONLY_F == 4096
    MIMO_LAUNCH_F(4096)
#elif MIMO_ONLY_F == 8192
    MIMO_LAUNCH_F(8192)
#endif
  }
  *found = false;
  return hipSuccess;
#else
  switch (k.F) {
    case 128: MIMO_LAUNCH_F(128)
    case 256: MIMO_LAUNCH_F(256)
    case 512: MIMO_LAUNCH_F(512)
    case 1024: MIMO_LAUNCH_F(1024)
    case 2048: MIMO_LAUNCH_F(2048)
    case 4096: MIMO_LAUNCH_F(4096)
    case 8192: MIMO_LAUNCH_F(8192)
    default: *found = false; return hipSuccess;
  }
#endif
#undef MIMO_LAUNCH_F
}

int validate_config(const mimo_config* c) {
  if (!c) return fail(MIMO_EINVAL, "null config");
  if (!is_pow2(c->n_fft) || c->n_fft < 128 || c->n_fft > 8192)
    return fail(MIMO_EINVAL, "n_fft must be a power of two in [128, 8192]");
  if (c->n_sub_carr < 4 || c->n_sub_carr % 4 || c->n_sub_carr > c->n_fft - 2)
    return fail(MIMO_EINVAL, "n_sub_carr must be a multiple of 4 in [4, n_fft - 2] (modulation.py:266-267 overlap)");
  const int L = (int)std::lround(std::sqrt((double)c->constel_size));
  if (L * L != c->constel_size || !is_pow2(c->constel_size) || c->constel_size < 4 || c->constel_size > 4096)
    return fail(MIMO_EINVAL, "Constellation size must be a power of some number, only square QAM supported.");
  if (c->n_ant < 1 || c->n_ant > 4096) return fail(MIMO_EINVAL, "n_ant must be in [1, 4096]");
  if (c->channel_kind < MIMO_CH_RAYLEIGH || c->channel_kind > MIMO_CH_TABLE)
    return fail(MIMO_EINVAL, "unknown channel_kind");
  if (c->channel_kind == MIMO_CH_TABLE && !c->chan_table)
    return fail(MIMO_EINVAL, "chan_table is required for MIMO_CH_TABLE");
  if (c->receiver_kind != MIMO_RX_CNC && c->receiver_kind != MIMO_RX_MCNC)
    return fail(MIMO_EINVAL, "unknown receiver_kind");
  if (!c->tx_pos) return fail(MIMO_EINVAL, "tx_pos is required");
  if (c->precision != MIMO_PREC_F64 && c->precision != MIMO_PREC_F32)
    return fail(MIMO_EINVAL, "precision must be MIMO_PREC_F64 or MIMO_PREC_F32");
  if (c->chan_replay_period < 0) return fail(MIMO_EINVAL, "chan_replay_period must be >= 0");
  if (c->chan_replay_period > 0 && c->channel_kind != MIMO_CH_RAYLEIGH)
    return fail(MIMO_EINVAL, "chan_replay_period applies to the Rayleigh channel only");
  return MIMO_OK;
}

int validate_point(const mimo_engine* e, const mimo_point* pt) {
  auto bad_kind = [](int k) { return k < MIMO_PA_NONE || k > MIMO_PA_TOI; };
  if (bad_kind(pt->pa_kind) || bad_kind(pt->cnc_pa_kind)) return fail(MIMO_EINVAL, "unknown PA kind");
  if ((pt->pa_kind == MIMO_PA_SOFTLIM || pt->pa_kind == MIMO_PA_RAPP) && !(pt->sat_pow > 0))
    return fail(MIMO_EINVAL, "sat_pow must be > 0");
  if (pt->pa_kind == MIMO_PA_RAPP && !(pt->p_hardness > 0)) return fail(MIMO_EINVAL, "p_hardness must be > 0");
  if (!(pt->cnc_alpha != 0)) return fail(MIMO_EINVAL, "cnc_alpha must be non-zero");
  if (pt->csi_eps >= 1.0) return fail(MIMO_EINVAL, "csi_eps must be < 1");
  if (pt->csi_eps >= 0 && e->cfg.n_ant > mimo::kMaxCsiAnt) return fail(MIMO_EINVAL, "CSI error supports n_ant <= 512");
  if (!(pt->array_alpha >= 0) || !std::isfinite(pt->array_alpha))
    return fail(MIMO_EINVAL, "array_alpha must be finite and >= 0");
  // the float32 F 8192 instance forms alpha by the library formula only (no polynomial to hold a constant)
  if (pt->array_alpha > 0 && e->cfg.precision == MIMO_PREC_F32 && e->cfg.n_fft == 8192)
    return fail(MIMO_EINVAL, "array_alpha needs float64 or n_fft <= 4096");
  return MIMO_OK;
}

// Per-point fields of the kernel parameters (the reference's per-point object state).
template <typename R>
void fill_point(mimo_engine* e, const mimo_point& pt, uint64_t seed, uint64_t first_trial,
                mimo::TrialParams<R>& p) {
  const mimo_config& c = e->cfg;
  const bool csi = pt.csi_eps >= 0;
  p.seed = seed;
  p.csi_seed = c.csi_seed ? c.csi_seed : seed;  // used by CH_TABLE + CSI only
  p.first_trial = first_trial;
  p.pa_kind = pt.pa_kind;
  p.cnc_pa_kind = pt.cnc_pa_kind;
  p.sat_tx = (R)pt.sat_pow;
  p.sqrt_sat_tx = (R)std::sqrt(std::max(pt.sat_pow, 0.0));
  p.inv_sat_tx = pt.sat_pow > 0 ? (R)(1.0 / pt.sat_pow) : R(0);
  p.rapp_p = (R)pt.p_hardness;
  p.toi_tx = (R)pt.toi_coeff;
  p.sat_cnc = (R)pt.cnc_sat_pow;
  p.sqrt_sat_cnc = (R)std::sqrt(std::max(pt.cnc_sat_pow, 0.0));
  p.inv_sat_cnc = pt.cnc_sat_pow > 0 ? (R)(1.0 / pt.cnc_sat_pow) : R(0);
  p.toi_cnc = (R)pt.cnc_toi_coeff;
  p.inv_alpha_cnc = (R)(1.0 / pt.cnc_alpha);
  p.alpha_c = (R)(std::pow(10.0, pt.ibo_db / 10.0) * c.n_sub_carr / c.n_ant);
  {
    const double g0sq = std::pow(10.0, pt.ibo_db / 10.0);
    uint64_t key;
    std::memcpy(&key, &g0sq, sizeof key);
    auto it = e->alpha_fits.find(key);
    if (it == e->alpha_fits.end()) {
      if (e->alpha_fits.size() >= 4096) e->alpha_fits.clear();
      it = e->alpha_fits.emplace(key, fit_alpha(g0sq)).first;
    }
    const AlphaFit& af = it->second;
    for (int i = 0; i < 9; ++i) p.apoly[i] = (R)af.apoly[i];
    p.alpha_xlim = (R)af.xlim;
    for (int k = 0; k < 19; ++k) p.amono64[k] = af.amono[k];
  }
  if (pt.array_alpha > 0) {
    // one fixed gain for every antenna: the kernel's alpha polynomial made the constant over
    // the whole range (the Horner sums then return it exactly)
    for (int i = 0; i < 9; ++i) p.apoly[i] = i == 0 ? (R)pt.array_alpha : R(0);
    for (int k = 0; k < 19; ++k) p.amono64[k] = k == 0 ? pt.array_alpha : 0.0;
    p.alpha_xlim = std::numeric_limits<R>::max();
  }
  p.es_over_snr = (R)(pt.avg_symbol_power / std::pow(10.0, pt.snr_db / 10.0));
  p.csi_a = csi ? (R)std::sqrt(1.0 - pt.csi_eps * pt.csi_eps) : R(1);
  p.csi_b = csi ? (R)pt.csi_eps : R(0);
}

template <typename T>
int ensure_cap(T*& ptr, size_t& cap, size_t need) {
  if (need <= cap) return MIMO_OK;
  if (ptr) HIP_TRY(hipFree(ptr));
  ptr = nullptr;
  HIP_TRY(hipMalloc(&ptr, need * sizeof(T)));
  cap = need;
  return MIMO_OK;
}

int ensure_device(mimo_engine* e) {
  if (e->ready) return MIMO_OK;
  if (e->cfg.device >= 0) HIP_TRY(hipSetDevice(e->cfg.device));
  HIP_TRY(hipGetDevice(&e->device));
  HIP_TRY(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
  HIP_TRY(hipEventCreate(&e->ev0));
  HIP_TRY(hipEventCreate(&e->ev1));
  const int F = e->cfg.n_fft, S = e->cfg.n_sub_carr, A = e->cfg.n_ant;
  // team-FFT stage twiddles per team size (team_fft.h plan), computed in double:
  // stage s, entry [r][jm] = exp(-j 2 pi e / F) with e = jm r F / (NS R)
  auto twiddles_of = [](int F, int T, auto cvt) {
    const int P = F / T;
    using V = decltype(cvt(0.0, 0.0));
    std::vector<V> tw(std::max(1, mimo::fft_tw_total(F, P)), cvt(0.0, 0.0));
    for (int st = 1; st < mimo::fft_nst(F, P); ++st) {
      const int NS = 1 << mimo::fft_bits_before(F, P, st), R = 1 << mimo::fft_bits(F, P, st);
      V* blk = tw.data() + mimo::fft_tw_off(F, P, st);
      for (int r = 0; r < R; ++r)
        for (int jm = 0; jm < NS; ++jm) {
          const long e_idx = (long)jm * r * (F / (NS * R));
          const double ang = -2.0 * M_PI * (double)e_idx / (double)F;
          blk[r * NS + jm] = cvt(std::cos(ang), std::sin(ang));
        }
    }
    return tw;
  };
  // cot-tan constants of the twiddled stages (team_fft.h dft8_ct / dft16_ct), appended to a
  // stage table: (cos a, tan a) per (stage, row, lane); cos is never exactly 0 in double
  // (cos(pi/2) = 6.1e-17), so tan stays finite
  // (appended for every instance; the kernels that do not run cot-tan stages never read them)
  auto append_ct = [](auto& tw, int Fs, int P, auto cvt) {
    for (int st = 1; st < mimo::fft_nst(Fs, P); ++st) {
      const int NS = 1 << mimo::fft_bits_before(Fs, P, st), R = 1 << mimo::fft_bits(Fs, P, st);
      for (int q = 0; q < mimo::ct_rows(R); ++q)
        for (int jm = 0; jm < NS; ++jm) {
          const double a = 2.0 * M_PI * mimo::ct_rev(R, NS, jm, q), c = std::cos(a);
          tw.push_back(cvt(c, std::sin(a) / c));
        }
    }
  };
  auto twiddles = [&](int T, auto cvt) {
    auto tw = twiddles_of(F, T, cvt);
    tw.resize(std::max(1, mimo::fft_tw_total(F, F / T)));
    if (F / T >= 2) append_ct(tw, F, F / T, cvt);
    return tw;
  };
  auto to_f32 = [](double c, double s) { return make_float2((float)c, (float)s); };
  auto to_f64 = [](double c, double s) { return make_double2(c, s); };
  std::vector<float2> tws[2] = {twiddles(mimo::team_size(F), to_f32), twiddles(mimo::alt_team_size(F), to_f32)};
  std::vector<double2> tw64 = twiddles(mimo::team_size64(F), to_f64);
  // split FFT (split_fft.h): the F/2-point sub-transform's table, its cot-tan region, then
  // the radix-2 stage's (cos a, tan a), a = -2 pi n / F, n < F/2.  At n = F/4 the pair is
  // (6.1e-17, -1.6e16): c t rounds to sin a, and the product form c (u.x - t u.y) keeps full
  // precision there (tests/test_fft_split.py, near the quarter turn)
  if (mimo::split_fft_used(F, mimo::team_size64(F), true)) {
    const int T = mimo::team_size64(F), P = F / T;
    tw64 = twiddles_of(F / 2, T / 2, to_f64);
    tw64.resize(mimo::fft_tw_total(F / 2, P));
    if (mimo::kSplitCt) append_ct(tw64, F / 2, P, to_f64);
    for (int n = 0; n < F / 2; ++n) {
      const double a = -2.0 * M_PI * (double)n / (double)F, c = std::cos(a);
      tw64.push_back(make_double2(c, std::sin(a) / c));
    }
    if ((int)tw64.size() != mimo::split_fft_tw_total(F, T)) return MIMO_ENOKERNEL;  // table and kernel disagree
  }
  // wave-split FFT (wave_fft.h): the one-wave sub-transform's stages, then exp(-j 2 pi n / F)
  auto wave_twiddles = [&](int T, auto cvt) {
    auto tw = twiddles_of(mimo::wave_fft_fw(F, T), 64, cvt);
    tw.resize(mimo::wave_fft_tw_inter(F, T));
    for (int n = 0; n < F; ++n) {
      const double ang = -2.0 * M_PI * (double)n / (double)F;
      tw.push_back(cvt(std::cos(ang), std::sin(ang)));
    }
    append_ct(tw, mimo::wave_fft_fw(F, T), F / T, cvt);  // the sub-transforms' cot-tan region
    return tw;
  };
  std::vector<double2> twave64;
  std::vector<float2> twave32;
  if (mimo::wave_fft_used(F, mimo::team_size64(F), true)) twave64 = wave_twiddles(mimo::team_size64(F), to_f64);
  if (mimo::wave_fft_used(F, mimo::team_size(F), false)) twave32 = wave_twiddles(mimo::team_size(F), to_f32);
  // in-band sub-carrier k -> bin (modulation.py:266-267)
  std::vector<float> f_rel(S);
  std::vector<double> f_rel64(S), f_over_c(S);
  const double fc = e->freqs[0];  // bin 0 = centre frequency
  for (int k = 0; k < S; ++k) {
    const int bin = k < S / 2 ? F - S / 2 + k : k - S / 2 + 1;
    const double f = e->freqs[bin];
    // table channels carry their full attenuation: nothing is factored out of the loops
    f_rel64[k] = e->cfg.channel_kind == MIMO_CH_TABLE ? 1.0 : fc / f;
    f_rel[k] = (float)f_rel64[k];
    f_over_c[k] = f / kSpeedOfLight;
  }
  // Rayleigh FSPL at the nominal RX (channel.py:216-225), relative to the nearest antenna
  std::vector<double> dist(A);
  double dmin = 1e300;
  for (int a = 0; a < A; ++a) {
    const double dx = e->tx_pos[3 * a] - e->cfg.rx_pos[0], dy = e->tx_pos[3 * a + 1] - e->cfg.rx_pos[1],
                 dz = e->tx_pos[3 * a + 2] - e->cfg.rx_pos[2];
    dist[a] = std::sqrt(dx * dx + dy * dy + dz * dz);
    dmin = std::min(dmin, dist[a]);
  }
  e->d0 = dmin > 0 ? dmin : 1.0;
  std::vector<float> ant_rel(A);
  std::vector<double> ant_rel64(A);
  for (int a = 0; a < A; ++a) {
    ant_rel64[a] = e->d0 / dist[a];
    ant_rel[a] = (float)ant_rel64[a];
  }

  for (int v = 0; v < 2; ++v) {
    HIP_TRY(hipMalloc(&e->d_tw[v], sizeof(float2) * tws[v].size()));
    HIP_TRY(hipMemcpy(e->d_tw[v], tws[v].data(), sizeof(float2) * tws[v].size(), hipMemcpyHostToDevice));
  }
  if (!e->chan_inband.empty()) {
    const size_t n = e->chan_inband.size() / 2;
    std::vector<float2> t32(n);
    for (size_t i = 0; i < n; ++i) t32[i] = make_float2((float)e->chan_inband[2 * i], (float)e->chan_inband[2 * i + 1]);
    HIP_TRY(hipMalloc(&e->d_tab32, sizeof(float2) * n));
    HIP_TRY(hipMalloc(&e->d_tab64, sizeof(double2) * n));
    HIP_TRY(hipMemcpy(e->d_tab32, t32.data(), sizeof(float2) * n, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(e->d_tab64, e->chan_inband.data(), sizeof(double2) * n, hipMemcpyHostToDevice));
  }
  const std::vector<double2> lut = lut64_table();
  HIP_TRY(hipMalloc(&e->d_lut64, sizeof(double2) * lut.size()));
  HIP_TRY(hipMemcpy(e->d_lut64, lut.data(), sizeof(double2) * lut.size(), hipMemcpyHostToDevice));
  HIP_TRY(hipMalloc(&e->d_tw64, sizeof(double2) * tw64.size()));
  HIP_TRY(hipMemcpy(e->d_tw64, tw64.data(), sizeof(double2) * tw64.size(), hipMemcpyHostToDevice));
  if (!twave64.empty()) {
    HIP_TRY(hipMalloc(&e->d_twave64, sizeof(double2) * twave64.size()));
    HIP_TRY(hipMemcpy(e->d_twave64, twave64.data(), sizeof(double2) * twave64.size(), hipMemcpyHostToDevice));
  }
  if (!twave32.empty()) {
    HIP_TRY(hipMalloc(&e->d_twave32, sizeof(float2) * twave32.size()));
    HIP_TRY(hipMemcpy(e->d_twave32, twave32.data(), sizeof(float2) * twave32.size(), hipMemcpyHostToDevice));
  }
  HIP_TRY(hipMalloc(&e->d_f_rel64, sizeof(double) * S));
  HIP_TRY(hipMalloc(&e->d_ant_rel64, sizeof(double) * A));
  HIP_TRY(hipMemcpy(e->d_f_rel64, f_rel64.data(), sizeof(double) * S, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(e->d_ant_rel64, ant_rel64.data(), sizeof(double) * A, hipMemcpyHostToDevice));
  HIP_TRY(hipMalloc(&e->d_f_rel, sizeof(float) * S));
  HIP_TRY(hipMalloc(&e->d_f_over_c, sizeof(double) * S));
  HIP_TRY(hipMalloc(&e->d_ant_rel, sizeof(float) * A));
  HIP_TRY(hipMalloc(&e->d_tx_pos, sizeof(double) * 3 * A));
  HIP_TRY(hipMemcpy(e->d_f_rel, f_rel.data(), sizeof(float) * S, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(e->d_f_over_c, f_over_c.data(), sizeof(double) * S, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(e->d_ant_rel, ant_rel.data(), sizeof(float) * A, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(e->d_tx_pos, e->tx_pos.data(), sizeof(double) * 3 * A, hipMemcpyHostToDevice));
  e->ready = true;
  return MIMO_OK;
}

}  // namespace

extern "C" {

int32_t mimo_abi_version(void) { return MIMO_ABI_VERSION; }
const char* mimo_last_error(void) { return g_err.c_str(); }

int32_t mimo_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

mimo_engine* mimo_engine_create(const mimo_config* cfg) {
  if (validate_config(cfg) != MIMO_OK) return nullptr;
  auto* e = new mimo_engine();
  e->cfg = *cfg;
  const int A = cfg->n_ant, F = cfg->n_fft;
  e->tx_pos.assign(cfg->tx_pos, cfg->tx_pos + 3 * A);
  e->freqs.resize(F);
  if (cfg->carrier_freqs) {
    std::copy(cfg->carrier_freqs, cfg->carrier_freqs + F, e->freqs.begin());
  } else {
    fail(MIMO_EINVAL, "carrier_freqs is required");
    delete e;
    return nullptr;
  }
  e->cfg.tx_pos = nullptr;
  e->cfg.carrier_freqs = nullptr;
  if (cfg->channel_kind == MIMO_CH_TABLE) {  // keep the in-band columns, bins b(k) (modulation.py:266-267)
    const int S = cfg->n_sub_carr;
    e->chan_inband.resize((size_t)A * S * 2);
    for (int a = 0; a < A; ++a)
      for (int k = 0; k < S; ++k) {
        const int bin = k < S / 2 ? F - S / 2 + k : k - S / 2 + 1;
        e->chan_inband[((size_t)a * S + k) * 2] = cfg->chan_table[((size_t)a * F + bin) * 2];
        e->chan_inband[((size_t)a * S + k) * 2 + 1] = cfg->chan_table[((size_t)a * F + bin) * 2 + 1];
      }
  }
  e->cfg.chan_table = nullptr;
  return e;
}

int32_t mimo_engine_set_point(mimo_engine* e, const mimo_point* pt) {
  if (!e || !pt) return fail(MIMO_EINVAL, "null argument");
  if (int rc = validate_point(e, pt)) return rc;
  e->pt = *pt;
  e->have_point = true;
  return MIMO_OK;
}

}  // extern "C"

namespace {

// Runs n_points grid points of one system in as few launches as possible: every point's
// trials become a contiguous range of blocks of one launch (split across launches only
// beyond kChunk blocks), and a segmented reduction sums each point's counts.
int run_points(mimo_engine* e, int n_points, const mimo_point* pts, const uint64_t* seeds,
               const uint64_t* first_trial, const uint64_t* n_trials, const int32_t* iters, int32_t n_iters,
               int32_t incl_clean, uint64_t* err_out, uint64_t* bits_out, uint32_t* per_trial) {
  if (n_points < 0) return fail(MIMO_EINVAL, "n_points must be >= 0");
  if (n_iters < 1 || !iters) return fail(MIMO_EINVAL, "at least one iteration index is required");
  uint32_t rec_mask = 0;
  int max_iter = -1;
  for (int i = 0; i < n_iters; ++i) {
    if (iters[i] < 0 || iters[i] > 31) return fail(MIMO_EINVAL, "iterations must be in [0, 31]");
    if (i && iters[i] <= iters[i - 1]) return fail(MIMO_EINVAL, "iterations must be sorted and unique");
    rec_mask |= 1u << iters[i];
    max_iter = std::max(max_iter, (int)iters[i]);
  }
  if (!err_out || !bits_out) return fail(MIMO_EINVAL, "null counters");
  if (n_points == 0) return MIMO_OK;
  if (!pts || !seeds || !first_trial || !n_trials) return fail(MIMO_EINVAL, "null point arrays");
  const int n_idx = n_iters + (incl_clean ? 1 : 0);
  const mimo_config& c = e->cfg;
  const bool csi = pts[0].csi_eps >= 0;
  for (int i = 0; i < n_points; ++i) {
    if (int rc = validate_point(e, &pts[i])) return rc;
    if ((pts[i].csi_eps >= 0) != csi) return fail(MIMO_EINVAL, "all points of one run must agree on CSI error on/off");
    if (n_trials[i] + first_trial[i] > (1ull << 32) || first_trial[i] >= (1ull << 32))
      return fail(MIMO_EINVAL, "trial index must fit 32 bits");
  }
  const mimo::InstanceKey key = select_instance(e, csi);
  if (int rc = ensure_device(e)) return rc;
  if (csi) {
    // the CSI instances add n_ant reals of dynamic LDS (the per-antenna power table) to their
    // static LDS: check the sum against the CU's LDS before launching (F 8192 holds
    // ~157 KiB statically, so A = 512 (4 KiB) is the edge)
    hipFuncAttributes fa{};
    bool found = false;
    hipError_t qe = key.f64 ? launch(key, dim3(0), e->stream, mimo::TrialParams<double>{}, &found, &fa)
                            : launch(key, dim3(0), e->stream, mimo::TrialParams<float>{}, &found, &fa);
    int lds_max = 0;
    if (found && qe == hipSuccess &&
        hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, e->device) == hipSuccess &&
        lds_max > 0) {
      const size_t need = fa.sharedSizeBytes + (size_t)c.n_ant * (key.f64 ? sizeof(double) : sizeof(float));
      if (need > (size_t)lds_max)
        return fail(MIMO_EINVAL, "CSI error at n_ant = " + std::to_string(c.n_ant) + " needs " + std::to_string(need) +
                                     " B of LDS per team (static " + std::to_string(fa.sharedSizeBytes) +
                                     " + the per-antenna table), the device has " + std::to_string(lds_max));
    }
  }
  if (!c.reroll_chan && (c.channel_kind == MIMO_CH_LOS || c.channel_kind == MIMO_CH_TWOPATH)) {
    // fixed RX: jitter span 0 around (x0, x0); only consistent when rx_y == rx_x
    // (table channels never use the RX position)
    if (c.rx_pos[1] != c.rx_pos[0]) return fail(MIMO_EINVAL, "reroll_chan=0 requires rx_pos[1] == rx_pos[0]");
  }
  char buf[160];
  snprintf(buf, sizeof buf, "F=%d T=%d slots=%d %s ch=%d csi=%d %s", key.F, key.T, key.nslot,
           key.aligned ? "aligned" : "generic", key.ch, (int)key.csi, key.f64 ? "f64" : "f32");
  e->desc = buf;

  // segments (point, first trial, count) packed into launches of <= kChunk blocks
  // Trials per launch: 2^20 (MIMO_MAX_LAUNCH_TRIALS lowers it, for tests of the splitting).
  uint64_t kChunk = 1ull << 20;
  if (const char* env = std::getenv("MIMO_MAX_LAUNCH_TRIALS")) {
    const uint64_t v = std::strtoull(env, nullptr, 10);
    if (v >= 1 && v < kChunk) kChunk = v;
  }
  struct Seg {
    int point;
    uint64_t first, n;
  };
  std::vector<std::vector<Seg>> launches(1);
  uint64_t fill = 0;
  for (int i = 0; i < n_points; ++i) {
    uint64_t done = 0;
    while (done < n_trials[i]) {
      if (fill == kChunk) {
        launches.emplace_back();
        fill = 0;
      }
      const uint64_t n = std::min(n_trials[i] - done, kChunk - fill);
      launches.back().push_back(Seg{i, first_trial[i] + done, n});
      done += n;
      fill += n;
    }
  }
  size_t max_seg = 0;
  for (auto& l : launches) max_seg = std::max(max_seg, l.size());
  if (int rc = ensure_cap(e->d_counts, e->counts_cap, (size_t)(1ull << 20) * n_idx)) return rc;
  if (int rc = ensure_cap(e->d_tot, e->tot_cap, (size_t)n_points * n_idx)) return rc;
  const size_t max_slices = max_seg + (size_t)(kChunk / kSlice) + 1;
  HIP_TRY(hipMemsetAsync(e->d_tot, 0, sizeof(unsigned long long) * n_points * n_idx, e->stream));
  double ms_total = 0.0;
  uint64_t rows_done = 0;

  auto run_as = [&](auto zero) -> int {
    using R = decltype(zero);
    using TP = mimo::TrialParams<R>;
    constexpr bool F64 = sizeof(R) == 8;
    TP base{};
    if constexpr (F64) {
      base.tw = e->d_tw64;
      base.tw_wave = e->d_twave64;
      base.ant_rel = e->d_ant_rel64;
      base.f_rel = e->d_f_rel64;
      base.chan_tab = e->d_tab64;
    } else {
      base.tw = e->d_tw[key.T == mimo::team_size(c.n_fft) ? 0 : 1];
      base.tw_wave = key.T == mimo::team_size(c.n_fft) ? e->d_twave32 : nullptr;
      base.ant_rel = e->d_ant_rel;
      base.f_rel = e->d_f_rel;
      base.chan_tab = e->d_tab32;
    }
    base.f_over_c = e->d_f_over_c;
    base.tx_pos = e->d_tx_pos;
    base.lut = e->d_lut64;
    base.n_ant = c.n_ant;
    base.n_sc = c.n_sub_carr;
    const int L = (int)std::lround(std::sqrt((double)c.constel_size));
    base.qam_l = L;
    base.half_bits = (int)std::lround(std::log2((double)L));
    base.label_mask = (uint32_t)c.constel_size - 1u;
    base.inv_vk0 = (R)((double)c.n_ant / c.n_sub_carr);
    base.inv_vk0_f = (R)((double)c.n_ant * c.n_fft / c.n_sub_carr);
    base.inv_sqrt_f = (R)(1.0 / std::sqrt((double)c.n_fft));
    base.receiver = c.receiver_kind;
    base.max_iter = max_iter;
    base.rec_mask = rec_mask;
    base.incl_clean = incl_clean ? 1 : 0;
    base.n_idx = n_idx;
    base.rx_x0 = c.rx_pos[0];
    base.rx_z = c.rx_pos[2];
    base.rx_var = c.reroll_chan ? c.rx_loc_var : 0.0;
    base.d0 = e->d0;
    base.ablate = 0;
#ifdef MIMO_ABLATION
    if (const char* env = std::getenv("MIMO_ABLATE")) base.ablate = (uint32_t)std::strtoul(env, nullptr, 0);
#endif
    base.counts = e->d_counts;
    base.chan_period = (uint32_t)std::max(0, c.chan_replay_period);
    // per-point parameter table (host), built once
    std::vector<TP> ptab(n_points, base);
    for (int i = 0; i < n_points; ++i) fill_point(e, pts[i], seeds[i], 0, ptab[i]);
    auto up16 = [](size_t b) { return (b + 15) & ~size_t(15); };
    const size_t o_start = up16(max_seg * sizeof(TP)), o_slice = o_start + up16((max_seg + 1) * sizeof(uint32_t)),
                 o_pof = o_slice + up16((max_slices + 1) * sizeof(uint32_t)),
                 blob = o_pof + up16(max_slices * sizeof(int32_t));
    if (int rc = ensure_cap(e->d_blob, e->blob_cap, blob)) return rc;
    if (blob > e->hblob_cap) {
      if (e->h_blob) HIP_TRY(hipHostFree(e->h_blob));
      e->h_blob = nullptr;
      HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&e->h_blob), blob, hipHostMallocDefault));
      e->hblob_cap = blob;
    }
    TP* seg_tab = reinterpret_cast<TP*>(e->h_blob);
    uint32_t* start = reinterpret_cast<uint32_t*>(e->h_blob + o_start);
    uint32_t* slice_first = reinterpret_cast<uint32_t*>(e->h_blob + o_slice);
    int32_t* point_of = reinterpret_cast<int32_t*>(e->h_blob + o_pof);
    for (auto& l : launches) {
      size_t nseg = 0, nsl = 0;
      start[0] = 0u;
      slice_first[0] = 0u;
      for (auto& sg : l) {
        TP q = ptab[sg.point];
        q.first_trial = sg.first;
        seg_tab[nseg] = q;
        const uint32_t b0 = start[nseg];
        start[++nseg] = b0 + (uint32_t)sg.n;
        for (uint32_t o = 0; o < (uint32_t)sg.n; o += kSlice) {
          slice_first[++nsl] = b0 + std::min<uint32_t>((uint32_t)sg.n, o + kSlice);
          point_of[nsl - 1] = sg.point;
        }
      }
      const uint32_t nb = start[nseg];
      if (nb == 0) continue;  // every point of the call has n_trials == 0: nothing to launch
      TP kp = base;
      kp.points = reinterpret_cast<const TP*>(e->d_blob);
      kp.point_start = reinterpret_cast<const uint32_t*>(e->d_blob + o_start);
      kp.n_points = (int)nseg;
      kp.seed = seg_tab[0].seed;  // unused by the kernel (read from the table)
      // the whole blob (unused tails included: one contiguous DMA)
      HIP_TRY(hipMemcpyAsync(e->d_blob, e->h_blob, o_pof + nsl * sizeof(int32_t), hipMemcpyHostToDevice, e->stream));
      HIP_TRY(hipEventRecord(e->ev0, e->stream));
      bool found = false;
      hipError_t le = launch(key, dim3(nb), e->stream, kp, &found);
      if (!found) return fail(MIMO_ENOKERNEL, std::string("no kernel instance for ") + buf);
      if (le != hipSuccess) return fail(MIMO_EHIP, std::string("trial kernel launch: ") + hipGetErrorString(le));
      HIP_TRY(hipEventRecord(e->ev1, e->stream));
      hipLaunchKernelGGL(reduce_counts, dim3((unsigned)nsl, n_idx), dim3(256), 0, e->stream, e->d_counts,
                         reinterpret_cast<const uint32_t*>(e->d_blob + o_slice),
                         reinterpret_cast<const int32_t*>(e->d_blob + o_pof), n_idx, e->d_tot);
      HIP_TRY(hipGetLastError());
      if (per_trial)
        HIP_TRY(hipMemcpyAsync(per_trial + rows_done * n_idx, e->d_counts, (size_t)nb * n_idx * sizeof(uint32_t),
                               hipMemcpyDeviceToHost, e->stream));
      rows_done += nb;
      // the host tables of the next launch are rewritten: wait for this one's copies
      HIP_TRY(hipEventSynchronize(e->ev1));
      float ms = 0.f;
      HIP_TRY(hipEventElapsedTime(&ms, e->ev0, e->ev1));
      ms_total += ms;
    }
    return MIMO_OK;
  };
  if (int rc = key.f64 ? run_as(0.0) : run_as(0.0f)) return rc;
  std::vector<unsigned long long> tot((size_t)n_points * n_idx);
  HIP_TRY(hipMemcpyAsync(tot.data(), e->d_tot, sizeof(unsigned long long) * tot.size(), hipMemcpyDeviceToHost,
                         e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  const uint64_t bits_per_trial = (uint64_t)c.n_sub_carr * (uint64_t)std::lround(std::log2((double)c.constel_size));
  for (int i = 0; i < n_points; ++i)
    for (int j = 0; j < n_idx; ++j) {
      err_out[(size_t)i * n_idx + j] += tot[(size_t)i * n_idx + j];
      bits_out[(size_t)i * n_idx + j] += bits_per_trial * n_trials[i];
    }
  e->last_ms = ms_total;
  return MIMO_OK;
}

}  // namespace

extern "C" {

int32_t mimo_engine_run(mimo_engine* e, uint64_t seed, uint64_t first_trial, uint64_t n_trials, const int32_t* iters,
                        int32_t n_iters, int32_t incl_clean, uint64_t* err_out, uint64_t* bits_out, uint32_t* per_trial) {
  if (!e) return fail(MIMO_EINVAL, "null engine");
  if (!e->have_point) return fail(MIMO_EINVAL, "mimo_engine_set_point was not called");
  if (n_trials == 0) {  // validate the iteration list, add nothing
    return run_points(e, 0, nullptr, nullptr, nullptr, nullptr, iters, n_iters, incl_clean, err_out, bits_out,
                      per_trial);
  }
  return run_points(e, 1, &e->pt, &seed, &first_trial, &n_trials, iters, n_iters, incl_clean, err_out, bits_out,
                    per_trial);
}

int32_t mimo_engine_run_points(mimo_engine* e, int32_t n_points, const mimo_point* points, const uint64_t* seeds,
                               const uint64_t* first_trial, const uint64_t* n_trials, const int32_t* iters,
                               int32_t n_iters, int32_t incl_clean, uint64_t* err_out, uint64_t* bits_out,
                               uint32_t* per_trial) {
  if (!e) return fail(MIMO_EINVAL, "null engine");
  return run_points(e, n_points, points, seeds, first_trial, n_trials, iters, n_iters, incl_clean, err_out, bits_out,
                    per_trial);
}

double mimo_engine_last_kernel_ms(const mimo_engine* e) { return e ? e->last_ms : 0.0; }

const char* mimo_engine_describe(const mimo_engine* e) {
  if (!e) return "";
  if (e->desc.empty()) {
    const mimo::InstanceKey k = select_instance(e, e->have_point && e->pt.csi_eps >= 0);
    char buf[160];
    snprintf(buf, sizeof buf, "F=%d T=%d slots=%d %s ch=%d csi=%d %s", k.F, k.T, k.nslot,
             k.aligned ? "aligned" : "generic", k.ch, (int)k.csi, k.f64 ? "f64" : "f32");
    const_cast<mimo_engine*>(e)->desc = buf;
  }
  return e->desc.c_str();
}

void mimo_engine_destroy(mimo_engine* e) {
  if (!e) return;
  if (e->ready) {
    (void)hipStreamSynchronize(e->stream);
    (void)hipFree(e->d_tw[0]);
    (void)hipFree(e->d_tw[1]);
    (void)hipFree(e->d_f_rel);
    (void)hipFree(e->d_tw64);
    if (e->d_twave64) (void)hipFree(e->d_twave64);
    if (e->d_twave32) (void)hipFree(e->d_twave32);
    (void)hipFree(e->d_lut64);
    if (e->d_tab32) (void)hipFree(e->d_tab32);
    if (e->d_tab64) (void)hipFree(e->d_tab64);
    (void)hipFree(e->d_f_rel64);
    (void)hipFree(e->d_ant_rel64);
    (void)hipFree(e->d_f_over_c);
    (void)hipFree(e->d_ant_rel);
    (void)hipFree(e->d_tx_pos);
    if (e->d_tot) (void)hipFree(e->d_tot);
    if (e->d_counts) (void)hipFree(e->d_counts);
    if (e->d_blob) (void)hipFree(e->d_blob);
    if (e->h_blob) (void)hipHostFree(e->h_blob);
    (void)hipEventDestroy(e->ev0);
    (void)hipEventDestroy(e->ev1);
    (void)hipStreamDestroy(e->stream);
  }
  delete e;
}

}  // extern "C"
