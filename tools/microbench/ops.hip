// Throughput of the instruction types the trial kernel leans on (gfx950).
// Each kernel runs 8 independent chains of one op per thread; all waves busy.
//   hipcc --offload-arch=gfx950 -O3 ops.hip -o ops && ./ops
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHAINS 8
#define ITERS 32768

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t seed) {
  uint32_t a[CHAINS];
  float f[CHAINS];
  float2 p2[CHAINS];
  double g[CHAINS];
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) {
    a[i] = seed + threadIdx.x * 7 + i;
    f[i] = (float)(threadIdx.x + i) * 1e-3f;
    p2[i] = make_float2(f[i], f[i] * 0.5f);
    g[i] = (double)f[i];
  }
  const uint32_t m = 0xD2511F53u + seed;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < CHAINS; ++i) {
      if constexpr (OP == 0) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "s"(m));
      if constexpr (OP == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "s"(m));
      if constexpr (OP == 2) {
        uint64_t r;
        uint64_t cc; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(r), "=s"(cc) : "v"(a[i]), "s"(m));
        a[i] = (uint32_t)r ^ (uint32_t)(r >> 32);
      }
      if constexpr (OP == 3) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "s"(m));
      if constexpr (OP == 4) asm volatile("v_fma_f32 %0, %0, %0, 1.0" : "+v"(f[i]));
      if constexpr (OP == 5) asm volatile("v_log_f32 %0, %0" : "+v"(f[i]));
      if constexpr (OP == 6) asm volatile("v_sin_f32 %0, %0" : "+v"(f[i]));
      if constexpr (OP == 7) {
        asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(p2[i]));
      }
      if constexpr (OP == 8) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "s"(m));
      if constexpr (OP == 9) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[i]) : "s"(m));
      if constexpr (OP == 10) asm volatile("v_fma_f64 %0, %0, %0, 1.0" : "+v"(g[i]));
      if constexpr (OP == 11) asm volatile("v_add_f64 %0, %0, 1.0" : "+v"(g[i]));
      if constexpr (OP == 12) asm volatile("v_mul_f64 %0, %0, %0" : "+v"(g[i]));
      if constexpr (OP == 13) asm volatile("v_rsq_f64 %0, %0" : "+v"(g[i]));
      if constexpr (OP == 14) asm volatile("v_mov_b64 %0, %0" : "+v"(g[i]));
      if constexpr (OP == 15) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(g[i]) : "v"(a[i]));
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) s += a[i] + __float_as_uint(f[i]) + __float_as_uint(p2[i].y) + (uint32_t)__double2loint(g[i]);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP>
void run(const char* name, uint32_t* d, int grid) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float ms = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<OP>, dim3(grid), dim3(256), 0, 0, d, 2u + rep);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float t = 0;
    hipEventElapsedTime(&t, e0, e1);
    if (rep) ms = t < ms ? t : ms;
  }
  const double wave_instr = (double)grid * 4 * ITERS * CHAINS;  // 4 waves per block
  // cycles per wave-instruction per SIMD at 2.4 GHz, 1024 SIMDs
  const double cyc = (ms * 1e-3) * 2.4e9 * 1024 / wave_instr;
  printf("%-22s %8.3f ms  %.2f SIMD-cycles per wave64 instruction\n", name, ms, cyc);
}

int main() {
  const int grid = 256 * 8;  // 8 blocks (32 waves) per CU
  uint32_t* d;
  hipMalloc(&d, sizeof(uint32_t) * grid * 256);
  run<4>("warmup fma", d, grid);
  run<3>("v_xor_b32", d, grid);
  run<4>("v_fma_f32", d, grid);
  run<7>("v_pk_fma_f32", d, grid);
  run<0>("v_mul_hi_u32", d, grid);
  run<1>("v_mul_lo_u32", d, grid);
  run<10>("v_fma_f64", d, grid);
  run<11>("v_add_f64", d, grid);
  run<12>("v_mul_f64", d, grid);
  run<13>("v_rsq_f64", d, grid);
  run<14>("v_mov_b64", d, grid);
  run<15>("v_cvt_f64_u32", d, grid);
  run<2>("v_mad_u64_u32(+xor)", d, grid);
  run<8>("v_mul_u32_u24", d, grid);
  run<9>("v_mul_hi_u32_u24", d, grid);
  run<5>("v_log_f32", d, grid);
  run<6>("v_sin_f32", d, grid);
  hipFree(d);
  return 0;
}
