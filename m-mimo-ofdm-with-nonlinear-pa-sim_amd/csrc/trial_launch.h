// Kernel-instance dispatch for the fused trial kernel (one object file per FFT size).
#pragma once
#include <hip/hip_runtime.h>

#include "trial_kernel.h"

namespace mimo {

// Team (workgroup) size per FFT size: 16 points per thread from F = 1024 up, one wave below.
constexpr int team_size(int F) { return F >= 1024 ? F / 16 : 64; }
// fp64 instances: 8 points per thread from F = 512 up (a complex double takes 4 VGPRs,
// so P = 8 holds the same 32 data registers as the fp32 team's P = 16), one wave below
// (16 points per thread below F = 8192 measured slower, profiles/r02/ab/ab64_p16_one_wave.json).
// F = 8192: 16 points per thread (T = 512, 2 waves/SIMD; its one 136 KiB exchange buffer
// allows one team per CU either way): 4 transform stages instead of 5, -8 % against the
// 1024-thread team once the Rapp gain stopped using the library log / exp
// (profiles/r03/ab8k/ab_micro_p16.json; it was +3.3 % before, profiles/r02/ab/ab8k_f64_team_pipe.json).
// F = 4096: 16 points per thread as well (T = 256, 3 stages, two 4-wave teams per CU at
// 80 KiB of LDS each): -29 % against the 512-thread wave-split team on the paper config
// (69.80 -> 49.66 ms per 32,768 trials, profiles/r03/ab_4k/).
constexpr int team_size64(int F) { return F >= 4096 ? F / 16 : F >= 512 ? F / 8 : 64; }
// Alternative team (8 points per thread: half the registers, 2x the waves, one more
// LDS exchange per transform), selectable with MIMO_TEAM=<T> for A/B measurements.
constexpr int alt_team_size(int F) { return F >= 1024 ? F / 8 : team_size(F); }

struct InstanceKey {
  int F, T, nslot;
  bool aligned;
  int ch;
  bool csi;
  bool f64;  // arithmetic type of the instance (TrialParams<double>)
};

// attr != null: return the instance's attributes (static LDS ...) instead of launching it
#define MIMO_DECLARE_LAUNCH(FV)                                                                           \
  hipError_t launch_trial_F##FV##_f32(const InstanceKey& k, dim3 grid, hipStream_t st,                    \
                                      const TrialParams<float>& p, bool* found,                           \
                                      hipFuncAttributes* attr = nullptr);                                 \
  hipError_t launch_trial_F##FV##_f64(const InstanceKey& k, dim3 grid, hipStream_t st,                    \
                                      const TrialParams<double>& p, bool* found,                          \
                                      hipFuncAttributes* attr = nullptr);
MIMO_DECLARE_LAUNCH(128)
MIMO_DECLARE_LAUNCH(256)
MIMO_DECLARE_LAUNCH(512)
MIMO_DECLARE_LAUNCH(1024)
MIMO_DECLARE_LAUNCH(2048)
MIMO_DECLARE_LAUNCH(4096)
MIMO_DECLARE_LAUNCH(8192)
#undef MIMO_DECLARE_LAUNCH

}  // namespace mimo
