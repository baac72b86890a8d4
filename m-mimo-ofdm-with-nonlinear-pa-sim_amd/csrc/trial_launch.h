// Kernel-instance dispatch for the fused trial kernel (one object file per FFT size).
#pragma once
#include <hip/hip_runtime.h>

#include "trial_kernel.h"

namespace mimo {

// Team (workgroup) size per FFT size: 16 points per thread from F = 1024 up, one wave below.
constexpr int team_size(int F) { return F >= 1024 ? F / 16 : 64; }
// Alternative team (8 points per thread: half the registers, 2x the waves, one more
// LDS exchange per transform), selectable with MIMO_TEAM=<T> for A/B measurements.
constexpr int alt_team_size(int F) { return F >= 1024 ? F / 8 : team_size(F); }

struct InstanceKey {
  int F, T, nslot;
  bool aligned;
  int ch;
  bool csi;
};

#define MIMO_DECLARE_LAUNCH(FV)                                                                  \
  hipError_t launch_trial_F##FV(const InstanceKey& k, dim3 grid, hipStream_t st, const TrialParams& p, \
                                bool* found);
MIMO_DECLARE_LAUNCH(128)
MIMO_DECLARE_LAUNCH(256)
MIMO_DECLARE_LAUNCH(512)
MIMO_DECLARE_LAUNCH(1024)
MIMO_DECLARE_LAUNCH(2048)
MIMO_DECLARE_LAUNCH(4096)
MIMO_DECLARE_LAUNCH(8192)
#undef MIMO_DECLARE_LAUNCH

}  // namespace mimo
