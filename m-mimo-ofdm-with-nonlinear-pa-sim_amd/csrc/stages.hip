// Fine-seam stage kernels (float64, caller-owned host arrays) for the Python object API
// mirror: OfdmQamModem, SoftLimiter/Rapp/ThirdOrderNonLin, AntennaArray precoding,
// Miso*Fd.propagate, Awgn, count_mismatched_bits, CncReceiver.  These are not the hot
// path (mimo_engine_run is); they give the object API the reference's float64 numerics
// (bit-exact on the QAM index path) on the GPU.
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>
#include <vector>

#include "../../include/mimo_engine.h"
#include "alpha_fit.h"
#include "philox.h"

namespace {

int sfail(int code, const std::string& m);

#define S_TRY(expr)                                                                               \
  do {                                                                                            \
    hipError_t _e = (expr);                                                                       \
    if (_e != hipSuccess) return sfail(MIMO_EHIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

bool pow2(long v) { return v > 0 && (v & (v - 1)) == 0; }
int qam_l(int M) {
  const int L = (int)std::lround(std::sqrt((double)M));
  return (L * L == M && pow2(M) && M >= 4 && M <= 4096) ? L : 0;
}

// RAII device buffer
struct DBuf {
  void* p = nullptr;
  hipError_t alloc(size_t n) { return hipMalloc(&p, n ? n : 1); }
  ~DBuf() {
    if (p) (void)hipFree(p);
  }
  template <typename T>
  T* as() { return reinterpret_cast<T*>(p); }
};

__device__ __forceinline__ uint32_t gray(uint32_t i) { return i ^ (i >> 1); }
__device__ __forceinline__ uint32_t gray_inv(uint32_t g) {
  g ^= g >> 1; g ^= g >> 2; g ^= g >> 4; g ^= g >> 8;
  return g;
}
// Per-axis slicer with the reference's lowest-label tie-break (modulation.py:75-76).
__device__ __forceinline__ uint32_t slice_axis_d(double x, int L) {
  const double q = (x + (double)L) * 0.5;
  const double fi = floor(q);
  long i = (long)fi;
  if (q == fi && i > 0 && i < L) i = gray((uint32_t)(i - 1)) < gray((uint32_t)i) ? i - 1 : i;
  i = i < 0 ? 0 : (i > L - 1 ? L - 1 : i);
  return gray((uint32_t)i);
}

__global__ void k_qam_map(int L, int hb, const int32_t* lab, int64_t n, double2* out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t l = (uint32_t)lab[i];
    const uint32_t ii = gray_inv(l >> hb), iq = gray_inv(l & ((1u << hb) - 1u));
    out[i] = make_double2(2.0 * ii - (L - 1), 2.0 * iq - (L - 1));
  }
}

__global__ void k_qam_slice(int L, int hb, const double2* in, int64_t n, int32_t* lab) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    lab[i] = (int32_t)((slice_axis_d(in[i].x, L) << hb) | slice_axis_d(in[i].y, L));
}

// soft_decoding (modulation.py:29-59)
__global__ void k_qam_llr(int M, int L, int hb, int nb, const double2* in, int64_t n, const double* nv, double* out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double2 z = in[i];
    for (int b = 0; b < nb; ++b) {
      double num = 0, den = 0;
      for (int m = 0; m < M; ++m) {
        const uint32_t ii = gray_inv((uint32_t)m >> hb), iq = gray_inv((uint32_t)m & ((1u << hb) - 1u));
        const double dx = z.x - (2.0 * ii - (L - 1)), dy = z.y - (2.0 * iq - (L - 1));
        const double e = exp(-(dx * dx + dy * dy) / nv[i]);
        if ((m >> b) & 1) num += e; else den += e;
      }
      out[i * nb + nb - 1 - b] = den == 0 ? INFINITY : log(fabs(num) / fabs(den));
    }
  }
}

// Batched ortho FFT, one workgroup per row, row in LDS (N <= 8192 doubles complex = 128 KiB).
__global__ void k_fft_rows(int N, int logN, int inverse, const double2* in, double2* out) {
  extern __shared__ double2 sm[];
  const double2* row = in + (size_t)blockIdx.x * N;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    const uint32_t r = __brev((uint32_t)i) >> (32 - logN);
    sm[r] = row[i];
  }
  __syncthreads();
  const double sgn = inverse ? 1.0 : -1.0;
  for (int len = 2; len <= N; len <<= 1) {
    const int half = len >> 1;
    for (int b = threadIdx.x; b < N / 2; b += blockDim.x) {
      const int grp = b / half, pos = b % half;
      const int i0 = grp * len + pos, i1 = i0 + half;
      double s, c;
      sincospi(sgn * 2.0 * pos / len, &s, &c);
      const double2 u = sm[i0], v = sm[i1];
      const double2 w = make_double2(v.x * c - v.y * s, v.x * s + v.y * c);
      sm[i0] = make_double2(u.x + w.x, u.y + w.y);
      sm[i1] = make_double2(u.x - w.x, u.y - w.y);
    }
    __syncthreads();
  }
  const double sc = 1.0 / sqrt((double)N);
  double2* orow = out + (size_t)blockIdx.x * N;
  for (int i = threadIdx.x; i < N; i += blockDim.x) orow[i] = make_double2(sm[i].x * sc, sm[i].y * sc);
}

// symbols [batch][S] -> zero-filled bins [batch][F] (modulation.py:265-267)
__global__ void k_to_bins(int F, int S, int64_t batch, const double2* sym, double2* fd) {
  const int64_t total = batch * F;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / F;
    const int n = (int)(i % F);
    double2 v = make_double2(0, 0);
    if (n >= F - S / 2) v = sym[b * S + (n - (F - S / 2))];
    else if (n >= 1 && n <= S / 2) v = sym[b * S + (n + S / 2 - 1)];
    fd[i] = v;
  }
}
// bins -> in-band symbols (modulation.py:292-293)
__global__ void k_from_bins(int F, int S, int64_t batch, const double2* fd, double2* sym) {
  const int64_t total = batch * S;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / S;
    const int k = (int)(i % S);
    const int n = k < S / 2 ? F - S / 2 + k : k - S / 2 + 1;
    sym[i] = fd[b * F + n];
  }
}
// prepend / drop cyclic prefix
__global__ void k_add_cp(int F, int cp, int64_t batch, const double2* td, double2* out) {
  const int64_t total = batch * (F + cp);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / (F + cp);
    const int n = (int)(i % (F + cp));
    out[i] = td[b * F + (n < cp ? F - cp + n : n - cp)];
  }
}
__global__ void k_drop_cp(int F, int cp, int64_t batch, const double2* in, double2* td) {
  const int64_t total = batch * F;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / F;
    td[i] = in[b * (F + cp) + cp + (i % F)];
  }
}

__global__ void k_pa(int kind, double sat, double p, double toi, const double2* in, int64_t n, double2* out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double2 x = in[i];
    const double pw = x.x * x.x + x.y * x.y;
    double sc = 1.0;
    if (kind == MIMO_PA_SOFTLIM) sc = pw <= sat ? 1.0 : sqrt(sat / (pw != 0 ? pw : 1.0));          // distortion.py:19
    else if (kind == MIMO_PA_RAPP) sc = 1.0 / pow(1.0 + pow(sqrt(pw) / sqrt(sat), 2 * p), 1.0 / (2 * p));  // :113
    else if (kind == MIMO_PA_TOI) sc = 1.0 - toi * pw;                                             // :211
    out[i] = make_double2(x.x * sc, x.y * sc);
  }
}

// MRT over rows: P[a][k] = conj(H[a][k]) / sqrt(sum_a |H[a][k]|^2)   (antenna_array.py:165-173)
__global__ void k_mrt(int A, int K, const double2* h, double2* p) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < K; k += gridDim.x * blockDim.x) {
    double s = 0;
    for (int a = 0; a < A; ++a) s += h[(size_t)a * K + k].x * h[(size_t)a * K + k].x + h[(size_t)a * K + k].y * h[(size_t)a * K + k].y;
    const double inv = 1.0 / sqrt(s);
    for (int a = 0; a < A; ++a) {
      const double2 v = h[(size_t)a * K + k];
      p[(size_t)a * K + k] = make_double2(v.x * inv, -v.y * inv);
    }
  }
}

// propagate: out[k] = sum_a H[a][k] Y[a][k]   (channel.py:287-290)
__global__ void k_combine(int A, int64_t K, const double2* h, const double2* y, double2* out) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < K; k += (int64_t)gridDim.x * blockDim.x) {
    double re = 0, im = 0;
    for (int a = 0; a < A; ++a) {
      const double2 hv = h[(size_t)a * K + k], yv = y[(size_t)a * K + k];
      re += hv.x * yv.x - hv.y * yv.y;
      im += hv.x * yv.y + hv.y * yv.x;
    }
    out[k] = make_double2(re, im);
  }
}

// Awgn.process (noise.py:56-83) with Philox draws: n = (x + jy) std / 2, x, y ~ N(0,1)
__global__ void k_awgn(uint64_t seed, uint64_t ctr, int64_t n, double std_, const double2* in, double2* out) {
  const mimo::Key key{(uint32_t)seed, (uint32_t)(seed >> 32)};
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint4 w = mimo::philox4x32_10(make_uint4((uint32_t)i, (uint32_t)ctr, 6u, (uint32_t)(ctr >> 32) ^ (uint32_t)(i >> 32)), key);
    const double u1 = ((double)w.x + 0.5) * 2.3283064365386963e-10, u2 = (double)w.y * 2.3283064365386963e-10;
    const double r = sqrt(-2.0 * log(u1));
    double s, c;
    sincospi(2.0 * u2, &s, &c);
    out[i] = make_double2(in[i].x + r * c * std_ * 0.5, in[i].y + r * s * std_ * 0.5);
  }
}

__global__ void k_count(const int64_t* a, const int64_t* b, int64_t n, unsigned long long* out) {
  unsigned long long acc = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    acc += (unsigned long long)(a[i] ^ b[i]);
  for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, acc);
}

// CNC distortion update: d = V / alpha - s_hat  (corrector.py:103-110)
__global__ void k_cnc_update(int S, int L, int hb, double inv_alpha, const double2* v, const int32_t* lab, double2* d) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < S; k += gridDim.x * blockDim.x) {
    const uint32_t l = (uint32_t)lab[k];
    const double sx = 2.0 * gray_inv(l >> hb) - (L - 1), sy = 2.0 * gray_inv(l & ((1u << hb) - 1u)) - (L - 1);
    d[k] = make_double2(v[k].x * inv_alpha - sx, v[k].y * inv_alpha - sy);
  }
}
__global__ void k_sub(int64_t n, const double2* a, const double2* b, double2* out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = make_double2(a[i].x - b[i].x, a[i].y - b[i].y);
}

dim3 grid_for(int64_t n) { return dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 4096))); }

int fft_device(int N, int64_t batch, int inverse, const double2* din, double2* dout) {
  if (!pow2(N) || N < 2 || N > 8192) return sfail(MIMO_EINVAL, "n_fft must be a power of two in [2, 8192]");
  int logN = 0;
  while ((1 << logN) < N) ++logN;
  const size_t lds = sizeof(double2) * N;
  S_TRY(hipFuncSetAttribute((const void*)k_fft_rows, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  if (batch > 0) hipLaunchKernelGGL(k_fft_rows, dim3((unsigned)batch), dim3(256), lds, 0, N, logN, inverse, din, dout);
  S_TRY(hipGetLastError());
  return MIMO_OK;
}

}  // namespace

namespace mimo {
void set_error(const std::string& m);  // engine.hip: one thread-local message for mimo_last_error()
}
namespace {
int sfail(int code, const std::string& m) {
  mimo::set_error(m);
  return code;
}
}  // namespace

extern "C" {

int32_t mimo_qam_map(int32_t M, const int32_t* labels, int64_t n, double* out_iq) {
  const int L = qam_l(M);
  if (!L) return sfail(MIMO_EINVAL, "Constellation size must be a power of some number, only square QAM supported.");
  int hb = 0;
  while ((1 << hb) < L) ++hb;
  DBuf dl, dout;
  S_TRY(dl.alloc(n * sizeof(int32_t)));
  S_TRY(dout.alloc(n * sizeof(double2)));
  S_TRY(hipMemcpy(dl.p, labels, n * sizeof(int32_t), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_qam_map, grid_for(n), dim3(256), 0, 0, L, hb, dl.as<int32_t>(), n, dout.as<double2>());
  S_TRY(hipGetLastError());
  S_TRY(hipMemcpy(out_iq, dout.p, n * sizeof(double2), hipMemcpyDeviceToHost));
  return MIMO_OK;
}

int32_t mimo_qam_slice(int32_t M, const double* in_iq, int64_t n, int32_t* labels_out) {
  const int L = qam_l(M);
  if (!L) return sfail(MIMO_EINVAL, "Constellation size must be a power of some number, only square QAM supported.");
  int hb = 0;
  while ((1 << hb) < L) ++hb;
  DBuf din, dl;
  S_TRY(din.alloc(n * sizeof(double2)));
  S_TRY(dl.alloc(n * sizeof(int32_t)));
  S_TRY(hipMemcpy(din.p, in_iq, n * sizeof(double2), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_qam_slice, grid_for(n), dim3(256), 0, 0, L, hb, din.as<double2>(), n, dl.as<int32_t>());
  S_TRY(hipGetLastError());
  S_TRY(hipMemcpy(labels_out, dl.p, n * sizeof(int32_t), hipMemcpyDeviceToHost));
  return MIMO_OK;
}

int32_t mimo_qam_llr(int32_t M, const double* in_iq, int64_t n, const double* noise_var, double* llr_out) {
  const int L = qam_l(M);
  if (!L) return sfail(MIMO_EINVAL, "Constellation size must be a power of some number, only square QAM supported.");
  int hb = 0;
  while ((1 << hb) < L) ++hb;
  const int nb = 2 * hb;
  DBuf din, dnv, dout;
  S_TRY(din.alloc(n * sizeof(double2)));
  S_TRY(dnv.alloc(n * sizeof(double)));
  S_TRY(dout.alloc(n * nb * sizeof(double)));
  S_TRY(hipMemcpy(din.p, in_iq, n * sizeof(double2), hipMemcpyHostToDevice));
  S_TRY(hipMemcpy(dnv.p, noise_var, n * sizeof(double), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_qam_llr, grid_for(n), dim3(256), 0, 0, M, L, hb, nb, din.as<double2>(), n, dnv.as<double>(),
                     dout.as<double>());
  S_TRY(hipGetLastError());
  S_TRY(hipMemcpy(llr_out, dout.p, n * nb * sizeof(double), hipMemcpyDeviceToHost));
  return MIMO_OK;
}

int32_t mimo_fft(int32_t N, int64_t batch, int32_t inverse, const double* in_iq, double* out_iq) {
  DBuf din, dout;
  const size_t bytes = (size_t)N * batch * sizeof(double2);
  S_TRY(din.alloc(bytes));
  S_TRY(dout.alloc(bytes));
  S_TRY(hipMemcpy(din.p, in_iq, bytes, hipMemcpyHostToDevice));
  if (int rc = fft_device(N, batch, inverse, din.as<double2>(), dout.as<double2>())) return rc;
  S_TRY(hipMemcpy(out_iq, dout.p, bytes, hipMemcpyDeviceToHost));
  return MIMO_OK;
}

int32_t mimo_ofdm_tx(int32_t F, int32_t S, int32_t cp, int64_t batch, const double* sym_iq, double* td_iq) {
  if (S < 2 || S > F - 2 || S % 2) return sfail(MIMO_EINVAL, "mod_symbols length must match n_sub_carr value");
  if (cp < 0 || cp > F) return sfail(MIMO_EINVAL, "bad cp_len");
  DBuf ds, dfd, dtd, dout;
  S_TRY(ds.alloc(batch * S * sizeof(double2)));
  S_TRY(dfd.alloc(batch * F * sizeof(double2)));
  S_TRY(dtd.alloc(batch * F * sizeof(double2)));
  S_TRY(dout.alloc(batch * (F + cp) * sizeof(double2)));
  S_TRY(hipMemcpy(ds.p, sym_iq, batch * S * sizeof(double2), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_to_bins, grid_for(batch * F), dim3(256), 0, 0, F, S, batch, ds.as<double2>(), dfd.as<double2>());
  if (int rc = fft_device(F, batch, 1, dfd.as<double2>(), dtd.as<double2>())) return rc;
  hipLaunchKernelGGL(k_add_cp, grid_for(batch * (F + cp)), dim3(256), 0, 0, F, cp, batch, dtd.as<double2>(),
                     dout.as<double2>());
  S_TRY(hipGetLastError());
  S_TRY(hipMemcpy(td_iq, dout.p, batch * (F + cp) * sizeof(double2), hipMemcpyDeviceToHost));
  return MIMO_OK;
}

int32_t mimo_ofdm_rx(int32_t F, int32_t S, int32_t cp, int64_t batch, const double* td_iq, double* sym_iq) {
  if (S < 2 || S > F - 2 || S % 2) return sfail(MIMO_EINVAL, "bad n_sub_carr");
  DBuf din, dtd, dfd, ds;
  S_TRY(din.alloc(batch * (F + cp) * sizeof(double2)));
  S_TRY(dtd.alloc(batch * F * sizeof(double2)));
  S_TRY(dfd.alloc(batch * F * sizeof(double2)));
  S_TRY(ds.alloc(batch * S * sizeof(double2)));
  S_TRY(hipMemcpy(din.p, td_iq, batch * (F + cp) * sizeof(double2), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_drop_cp, grid_for(batch * F), dim3(256), 0, 0, F, cp, batch, din.as<double2>(), dtd.as<double2>());
  if (int rc = fft_device(F, batch, 0, dtd.as<double2>(), dfd.as<double2>())) return rc;
  hipLaunchKernelGGL(k_from_bins, grid_for(batch * S), dim3(256), 0, 0, F, S, batch, dfd.as<double2>(), ds.as<double2>());
  S_TRY(hipGetLastError());
  S_TRY(hipMemcpy(sym_iq, ds.p, batch * S * sizeof(double2), hipMemcpyDeviceToHost));
  return MIMO_OK;
}

int32_t mimo_pa(int32_t kind, double sat, double p, double toi, const double* in_iq, int64_t n, double* out_iq) {
  if (kind < MIMO_PA_NONE || kind > MIMO_PA_TOI) return sfail(MIMO_EINVAL, "unknown PA kind");
  DBuf din, dout;
  S_TRY(din.alloc(n * sizeof(double2)));
  S_TRY(dout.alloc(n * sizeof(double2)));
  S_TRY(hipMemcpy(din.p, in_iq, n * sizeof(double2), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_pa, grid_for(n), dim3(256), 0, 0, kind, sat, p, toi, din.as<double2>(), n, dout.as<double2>());
  S_TRY(hipGetLastError());
  S_TRY(hipMemcpy(out_iq, dout.p, n * sizeof(double2), hipMemcpyDeviceToHost));
  return MIMO_OK;
}

// Modem.calc_alpha (modulation.py:178-189) through the trial kernel's segment table
// (alpha_fit.h alpha_seg).  alpha_seg wants a wave-uniform argument (scalar coefficient
// loads): one wave per element.
__global__ void k_calc_alpha(const double* g2, const double* tab, double* out) {
  const double a = mimo::alpha_seg(g2[blockIdx.x], tab);
  if (threadIdx.x == 0) out[blockIdx.x] = a;
}

int32_t mimo_calc_alpha(const double* ibo_db, int64_t n, double* out) {
  if (n < 0) return sfail(MIMO_EINVAL, "n < 0");
  if (n == 0) return MIMO_OK;
  if (n > (1 << 30)) return sfail(MIMO_EINVAL, "n too large");
  std::vector<double> g2(n);
  for (int64_t i = 0; i < n; ++i) g2[i] = std::pow(10.0, ibo_db[i] / 10.0);  // gamma^2, modulation.py:186
  const std::vector<double> tab = mimo::alpha_segment_table();
  DBuf dg, dt, dout;
  S_TRY(dg.alloc(n * sizeof(double)));
  S_TRY(dt.alloc(tab.size() * sizeof(double)));
  S_TRY(dout.alloc(n * sizeof(double)));
  S_TRY(hipMemcpy(dg.p, g2.data(), n * sizeof(double), hipMemcpyHostToDevice));
  S_TRY(hipMemcpy(dt.p, tab.data(), tab.size() * sizeof(double), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_calc_alpha, dim3((unsigned)n), dim3(64), 0, 0, dg.as<double>(), dt.as<double>(), dout.as<double>());
  S_TRY(hipGetLastError());
  S_TRY(hipMemcpy(out, dout.p, n * sizeof(double), hipMemcpyDeviceToHost));
  return MIMO_OK;
}

int32_t mimo_mrt_precode(int32_t A, int32_t K, const double* h_iq, double* p_iq) {
  DBuf dh, dp;
  const size_t bytes = (size_t)A * K * sizeof(double2);
  S_TRY(dh.alloc(bytes));
  S_TRY(dp.alloc(bytes));
  S_TRY(hipMemcpy(dh.p, h_iq, bytes, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_mrt, grid_for(K), dim3(256), 0, 0, A, K, dh.as<double2>(), dp.as<double2>());
  S_TRY(hipGetLastError());
  S_TRY(hipMemcpy(p_iq, dp.p, bytes, hipMemcpyDeviceToHost));
  return MIMO_OK;
}

int32_t mimo_combine(int32_t A, int64_t K, const double* h_iq, const double* y_iq, double* out_iq) {
  DBuf dh, dy, dout;
  const size_t bytes = (size_t)A * K * sizeof(double2);
  S_TRY(dh.alloc(bytes));
  S_TRY(dy.alloc(bytes));
  S_TRY(dout.alloc(K * sizeof(double2)));
  S_TRY(hipMemcpy(dh.p, h_iq, bytes, hipMemcpyHostToDevice));
  S_TRY(hipMemcpy(dy.p, y_iq, bytes, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_combine, grid_for(K), dim3(256), 0, 0, A, K, dh.as<double2>(), dy.as<double2>(), dout.as<double2>());
  S_TRY(hipGetLastError());
  S_TRY(hipMemcpy(out_iq, dout.p, K * sizeof(double2), hipMemcpyDeviceToHost));
  return MIMO_OK;
}

int32_t mimo_awgn(uint64_t seed, uint64_t counter, int64_t n, double noise_std, const double* in_iq, double* out_iq) {
  DBuf din, dout;
  S_TRY(din.alloc(n * sizeof(double2)));
  S_TRY(dout.alloc(n * sizeof(double2)));
  S_TRY(hipMemcpy(din.p, in_iq, n * sizeof(double2), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_awgn, grid_for(n), dim3(256), 0, 0, seed, counter, n, noise_std, din.as<double2>(),
                     dout.as<double2>());
  S_TRY(hipGetLastError());
  S_TRY(hipMemcpy(out_iq, dout.p, n * sizeof(double2), hipMemcpyDeviceToHost));
  return MIMO_OK;
}

int32_t mimo_count_bit_errors(const int64_t* a, const int64_t* b, int64_t n, int64_t* out) {
  DBuf da, db, dc;
  S_TRY(da.alloc(n * sizeof(int64_t)));
  S_TRY(db.alloc(n * sizeof(int64_t)));
  S_TRY(dc.alloc(sizeof(unsigned long long)));
  S_TRY(hipMemcpy(da.p, a, n * sizeof(int64_t), hipMemcpyHostToDevice));
  S_TRY(hipMemcpy(db.p, b, n * sizeof(int64_t), hipMemcpyHostToDevice));
  S_TRY(hipMemset(dc.p, 0, sizeof(unsigned long long)));
  hipLaunchKernelGGL(k_count, grid_for(n), dim3(256), 0, 0, da.as<int64_t>(), db.as<int64_t>(), n,
                     dc.as<unsigned long long>());
  S_TRY(hipGetLastError());
  unsigned long long c = 0;
  S_TRY(hipMemcpy(&c, dc.p, sizeof c, hipMemcpyDeviceToHost));
  *out = (int64_t)c;
  return MIMO_OK;
}

// CncReceiver.receive (corrector.py:52-112) for one in-band vector; labels_out is
// [n_iters][S] (the iterations listed, ascending); corrected_iq_out (return_bits=False,
// corrector.py:80-84) the slicer's input rx - d of those iterations, [n_iters][S] (re, im).
// Either output may be null.
int32_t mimo_cnc_receive_ex(int32_t M, int32_t F, int32_t S, int32_t pa_kind, double sat, double p, double toi,
                            double alpha, const int32_t* iters, int32_t n_iters, const double* in_sc_iq,
                            int32_t* labels_out, double* corrected_iq_out) {
  const int L = qam_l(M);
  if (!L) return sfail(MIMO_EINVAL, "Constellation size must be a power of some number, only square QAM supported.");
  if (n_iters < 1) return sfail(MIMO_EINVAL, "empty iteration list");
  int hb = 0;
  while ((1 << hb) < L) ++hb;
  int max_it = 0;
  for (int i = 0; i < n_iters; ++i) {
    if (iters[i] < 0 || (i && iters[i] <= iters[i - 1])) return sfail(MIMO_EINVAL, "iterations must be sorted, unique, >= 0");
    max_it = iters[i];
  }
  DBuf dz, dd, dv, dlab, dsym, dfd, dtd, dfd2;
  S_TRY(dz.alloc(S * sizeof(double2)));
  S_TRY(dd.alloc(S * sizeof(double2)));
  S_TRY(dv.alloc(S * sizeof(double2)));
  S_TRY(dlab.alloc(S * sizeof(int32_t)));
  S_TRY(dsym.alloc(S * sizeof(double2)));
  S_TRY(dfd.alloc(F * sizeof(double2)));
  S_TRY(dtd.alloc(F * sizeof(double2)));
  S_TRY(dfd2.alloc(F * sizeof(double2)));
  S_TRY(hipMemcpy(dz.p, in_sc_iq, S * sizeof(double2), hipMemcpyHostToDevice));
  S_TRY(hipMemset(dd.p, 0, S * sizeof(double2)));
  int out_i = 0;
  for (int it = 0; it <= max_it; ++it) {
    hipLaunchKernelGGL(k_sub, grid_for(S), dim3(256), 0, 0, (int64_t)S, dz.as<double2>(), dd.as<double2>(), dv.as<double2>());
    hipLaunchKernelGGL(k_qam_slice, grid_for(S), dim3(256), 0, 0, L, hb, dv.as<double2>(), (int64_t)S, dlab.as<int32_t>());
    S_TRY(hipGetLastError());
    if (out_i < n_iters && iters[out_i] == it) {
      if (labels_out)
        S_TRY(hipMemcpy(labels_out + (size_t)out_i * S, dlab.p, S * sizeof(int32_t), hipMemcpyDeviceToHost));
      if (corrected_iq_out)
        S_TRY(hipMemcpy(corrected_iq_out + (size_t)out_i * 2 * S, dv.p, S * sizeof(double2), hipMemcpyDeviceToHost));
      ++out_i;
    }
    if (it == max_it) break;
    hipLaunchKernelGGL(k_qam_map, grid_for(S), dim3(256), 0, 0, L, hb, dlab.as<int32_t>(), (int64_t)S, dsym.as<double2>());
    hipLaunchKernelGGL(k_to_bins, grid_for(F), dim3(256), 0, 0, F, S, (int64_t)1, dsym.as<double2>(), dfd.as<double2>());
    if (int rc = fft_device(F, 1, 1, dfd.as<double2>(), dtd.as<double2>())) return rc;
    hipLaunchKernelGGL(k_pa, grid_for(F), dim3(256), 0, 0, pa_kind, sat, p, toi, dtd.as<double2>(), (int64_t)F,
                       dtd.as<double2>());
    if (int rc = fft_device(F, 1, 0, dtd.as<double2>(), dfd2.as<double2>())) return rc;
    hipLaunchKernelGGL(k_from_bins, grid_for(S), dim3(256), 0, 0, F, S, (int64_t)1, dfd2.as<double2>(), dv.as<double2>());
    hipLaunchKernelGGL(k_cnc_update, grid_for(S), dim3(256), 0, 0, S, L, hb, 1.0 / alpha, dv.as<double2>(),
                       dlab.as<int32_t>(), dd.as<double2>());
    S_TRY(hipGetLastError());
  }
  S_TRY(hipDeviceSynchronize());
  return MIMO_OK;
}

int32_t mimo_cnc_receive(int32_t M, int32_t F, int32_t S, int32_t pa_kind, double sat, double p, double toi,
                         double alpha, const int32_t* iters, int32_t n_iters, const double* in_sc_iq,
                         int32_t* labels_out) {
  if (!labels_out) return sfail(MIMO_EINVAL, "null labels_out");
  return mimo_cnc_receive_ex(M, F, S, pa_kind, sat, p, toi, alpha, iters, n_iters, in_sc_iq, labels_out, nullptr);
}

}  // extern "C"
