// Instantiates the fused trial kernel for one FFT size (compiled once per -DINST_F=...).
#include "trial_launch.h"

#ifndef INST_F
#error "compile with -DINST_F=<fft size>"
#endif

#define MIMO_CAT2(a, b) a##b
#define MIMO_CAT(a, b) MIMO_CAT2(a, b)

namespace mimo {
namespace {

constexpr int kF = INST_F;

template <int T, int NSLOT, bool AL, int CH, bool CSI, int MINW>
hipError_t go(dim3 grid, hipStream_t st, const TrialParams& p) {
  hipLaunchKernelGGL((trial_kernel<kF, T, NSLOT, AL, CH, CSI, MINW>), grid, dim3(T), 0, st, p);
  return hipGetLastError();
}

template <int T, int NSLOT, bool AL, int MINW>
hipError_t by_channel(const InstanceKey& k, dim3 grid, hipStream_t st, const TrialParams& p, bool* found) {
  *found = true;
  switch (k.ch) {
    case CH_RAYLEIGH:
      return k.csi ? go<T, NSLOT, AL, CH_RAYLEIGH, true, MINW>(grid, st, p)
                   : go<T, NSLOT, AL, CH_RAYLEIGH, false, MINW>(grid, st, p);
    case CH_LOS:
      return k.csi ? go<T, NSLOT, AL, CH_LOS, true, MINW>(grid, st, p) : go<T, NSLOT, AL, CH_LOS, false, MINW>(grid, st, p);
    case CH_TWOPATH:
      return k.csi ? go<T, NSLOT, AL, CH_TWOPATH, true, MINW>(grid, st, p)
                   : go<T, NSLOT, AL, CH_TWOPATH, false, MINW>(grid, st, p);
    default:
      *found = false;
      return hipSuccess;
  }
}

// Occupancy target (waves per SIMD) by points per thread: 16 points fit 2 waves/SIMD,
// 8 points fit 4 (measured with -Rpass-analysis=kernel-resource-usage, no spills).
constexpr int minw_for(int P) { return P >= 16 ? 2 : 4; }

template <int T>
hipError_t by_team(const InstanceKey& k, dim3 grid, hipStream_t st, const TrialParams& p, bool* found) {
  constexpr int P = kF / T;
  constexpr int MW = minw_for(P);
  if (k.aligned) {
    if constexpr (8 < P) {
      if (k.nslot == 8) return by_channel<T, 8, true, MW>(k, grid, st, p, found);
    }
    if constexpr (4 < P) {
      if (k.nslot == 4) return by_channel<T, 4, true, MW>(k, grid, st, p, found);
    }
    return hipSuccess;
  }
  if (k.nslot != P) return hipSuccess;
  return by_channel<T, P, false, 2>(k, grid, st, p, found);
}

}  // namespace

hipError_t MIMO_CAT(launch_trial_F, INST_F)(const InstanceKey& k, dim3 grid, hipStream_t st, const TrialParams& p,
                                            bool* found) {
  *found = false;
  if (k.F != kF) return hipSuccess;
  if (k.T == team_size(kF)) return by_team<team_size(kF)>(k, grid, st, p, found);
  if constexpr (alt_team_size(kF) != team_size(kF)) {
    if (k.T == alt_team_size(kF)) return by_team<alt_team_size(kF)>(k, grid, st, p, found);
  }
  return hipSuccess;
}

}  // namespace mimo
