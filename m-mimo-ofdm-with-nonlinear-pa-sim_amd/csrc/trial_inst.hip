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
constexpr int kT = team_size(kF);
constexpr int kP = kF / kT;

template <int NSLOT, bool AL, int CH, bool CSI, int MINW>
hipError_t go(dim3 grid, hipStream_t st, const TrialParams& p) {
  hipLaunchKernelGGL((trial_kernel<kF, kT, NSLOT, AL, CH, CSI, MINW>), grid, dim3(kT), 0, st, p);
  return hipGetLastError();
}

template <int NSLOT, bool AL, int MINW>
hipError_t by_channel(const InstanceKey& k, dim3 grid, hipStream_t st, const TrialParams& p, bool* found) {
  *found = true;
  switch (k.ch) {
    case CH_RAYLEIGH:
      return k.csi ? go<NSLOT, AL, CH_RAYLEIGH, true, MINW>(grid, st, p) : go<NSLOT, AL, CH_RAYLEIGH, false, MINW>(grid, st, p);
    case CH_LOS:
      return k.csi ? go<NSLOT, AL, CH_LOS, true, MINW>(grid, st, p) : go<NSLOT, AL, CH_LOS, false, MINW>(grid, st, p);
    case CH_TWOPATH:
      return k.csi ? go<NSLOT, AL, CH_TWOPATH, true, MINW>(grid, st, p) : go<NSLOT, AL, CH_TWOPATH, false, MINW>(grid, st, p);
    default:
      *found = false;
      return hipSuccess;
  }
}

}  // namespace

hipError_t MIMO_CAT(launch_trial_F, INST_F)(const InstanceKey& k, dim3 grid, hipStream_t st, const TrialParams& p,
                                            bool* found) {
  *found = false;
  if (k.F != kF || k.T != kT) return hipSuccess;
  if (k.aligned) {
    if constexpr (8 < kP) {
      if (k.nslot == 8) return by_channel<8, true, 2>(k, grid, st, p, found);
    }
    if constexpr (4 < kP) {
      if (k.nslot == 4) return by_channel<4, true, 2>(k, grid, st, p, found);
    }
    return hipSuccess;
  }
  if (k.nslot != kP) return hipSuccess;
  return by_channel<kP, false, 2>(k, grid, st, p, found);
}

}  // namespace mimo
