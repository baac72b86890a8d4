// Instruction count of one team-FFT transform (tools/loop_hist.py-style inspection):
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -fno-slp-vectorize -I<csrc> -S tools/fft_only.hip
#include "team_fft.h"
#ifndef XF
#define XF 2048
#endif
#ifndef XT
#define XT 128
#endif
using FFT = mimo::TeamFft<XF, XT, 1>;
__global__ __launch_bounds__(XT) void fft_only(float2* io, const float2* tw) {
  __shared__ float2 lds[FFT::LDS_TOTAL];
  float2 d[FFT::P];
  for (int m = 0; m < FFT::P; ++m) d[m] = io[blockIdx.x * XF + threadIdx.x + XT * m];
  FFT::run<+1>(d, lds, tw, threadIdx.x);
  for (int m = 0; m < FFT::P; ++m) io[blockIdx.x * XF + threadIdx.x + XT * m] = d[m];
}
