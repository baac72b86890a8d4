// Accuracy of gfx950's f64 seed instructions (v_rsq_f64, v_rcp_f64, v_sqrt_f64) against
// long-double references on the host: decides how many Newton steps real.h needs.
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/f64_acc.hip -o /tmp/f64_acc && /tmp/f64_acc
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>

__global__ void seeds(const double* x, double* rsq, double* rcp, double* sq, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    rsq[i] = __builtin_amdgcn_rsq(x[i]);
    rcp[i] = __builtin_amdgcn_rcp(x[i]);
    sq[i] = __builtin_amdgcn_sqrt(x[i]);
  }
}

static double ulp_err(double got, long double ref) {
  const double r = (double)ref;
  const double u = std::nextafter(std::fabs(r), INFINITY) - std::fabs(r);
  return (double)(std::fabs((long double)got - ref) / (long double)u);
}

int main() {
  const int n = 1 << 22;
  std::vector<double> x(n), a(n), b(n), c(n);
  std::mt19937_64 g(7);
  std::uniform_real_distribution<double> e(-40.0, 40.0);
  for (int i = 0; i < n; ++i) x[i] = std::ldexp(1.0 + (double)(g() >> 11) * 0x1p-53, (int)e(g));
  double *dx, *da, *db, *dc;
  hipMalloc(&dx, n * 8); hipMalloc(&da, n * 8); hipMalloc(&db, n * 8); hipMalloc(&dc, n * 8);
  hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  seeds<<<n / 256, 256>>>(dx, da, db, dc, n);
  hipMemcpy(a.data(), da, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(b.data(), db, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(c.data(), dc, n * 8, hipMemcpyDeviceToHost);
  double m1 = 0, m2 = 0, m3 = 0;
  for (int i = 0; i < n; ++i) {
    const long double xi = x[i];
    m1 = std::fmax(m1, ulp_err(a[i], 1.0L / std::sqrt(xi)));
    m2 = std::fmax(m2, ulp_err(b[i], 1.0L / xi));
    m3 = std::fmax(m3, ulp_err(c[i], std::sqrt(xi)));
  }
  printf("{\"v_rsq_f64_max_ulp\": %.4g, \"v_rcp_f64_max_ulp\": %.4g, \"v_sqrt_f64_max_ulp\": %.4g, \"samples\": %d}\n",
         m1, m2, m3, n);
  return 0;
}
