// Instantiates the fused trial kernel for one FFT size and arithmetic type
// (compiled once per -DINST_F=<size> -DINST_F64=<0|1>).
#include <type_traits>

#include "trial_launch.h"

#ifndef INST_F
#error "compile with -DINST_F=<fft size>"
#endif
#ifndef INST_F64
#define INST_F64 0
#endif

#define MIMO_CAT2(a, b) a##b
#define MIMO_CAT(a, b) MIMO_CAT2(a, b)

namespace mimo {
namespace {

constexpr int kF = INST_F;
constexpr bool kF64 = INST_F64 != 0;
using Real = std::conditional_t<kF64, double, float>;

// Occupancy profile per instance (see trial_kernel): waves/SIMD target, exchange buffers,
// symbols in LDS.  Measured on MI355X (tools/ab_libs.py; DESIGN.md §3 has the A/Bs):
//  - fp64 up to F = 2048: 3 waves/SIMD (<= 168 VGPRs), one exchange buffer, the symbols
//    rebuilt per antenna from packed lattice levels (no symbols in LDS), 3 teams per CU.
//  - fp64 F = 4096: the 256-thread 16-point team, 2 waves/SIMD, one buffer, 2 teams/CU.
//  - fp64 F = 8192: the 512-thread 16-point team, 2 waves/SIMD, one team per CU.
//  - fp32 aligned, 16 points/thread, F <= 4096: 3 waves/SIMD with one exchange buffer and
//    the weighted symbols in LDS (F = 2048: 25 KiB / team).
//  - fp32 aligned, 8 points/thread: 4 waves/SIMD fit in 128 VGPRs with two buffers.
//  - generic (unaligned band): symbols in LDS to limit spills.
struct Profile {
  int minw, nbuf;
  bool symw_lds;
};
constexpr Profile profile_for(int T, bool aligned, int ch) {
  const int P = kF / T;
  if (kF64 && kF >= 8192) return Profile{2, 1, false};  // 136 KiB exchange buffer: one team per CU (T = 512: 2 waves/SIMD)
  // fp64 up to F 2048: 3 waves/SIMD (168 VGPRs; the symbols rebuilt from the labels and
  // |Hhat|^2 after the FFT, so 49.5 KiB of LDS per 256-thread team and 3 teams per CU):
  // -8.5 % at config 2 (profiles/r03/ab_w3/).
  if (kF64 && kF <= 2048) return Profile{MIMO_W64_2048, 1, false};
  if (kF64 && kF == 4096) return Profile{2, 1, false};  // 16-point team, symbols from levels: 2 teams/CU
  if (kF64) return Profile{2, 1, true};
  if (!aligned) return Profile{2, kF >= 4096 ? 1 : 2, true};  // one buffer from F = 4096: 2 teams/CU
  if (P < 16) return Profile{4, 2, false};
  if (kF <= 4096) return Profile{3, 1, true};
  return Profile{2, 2, false};
}

// attr != null: no launch, the instance's attributes instead (its static LDS, which the
// engine checks with the CSI table's dynamic LDS against the device limit before a launch)
template <int T, int NSLOT, bool AL, int CH, bool CSI>
hipError_t go(dim3 grid, hipStream_t st, const TrialParams<Real>& p, hipFuncAttributes* attr) {
  constexpr Profile pr = profile_for(T, AL, CH);
  auto* kern = &trial_kernel<Real, kF, T, NSLOT, AL, CH, CSI, pr.minw, pr.nbuf, pr.symw_lds>;
  if (attr) return hipFuncGetAttributes(attr, reinterpret_cast<const void*>(kern));
  // CSI: the per-antenna power table is dynamic LDS, A reals (trial_kernel pw_csi)
  const size_t dyn = CSI ? sizeof(Real) * (size_t)p.n_ant : 0;
  hipLaunchKernelGGL(kern, grid, dim3(T), dyn, st, p);
  return hipGetLastError();
}

template <int T, int NSLOT, bool AL>
hipError_t by_channel(const InstanceKey& k, dim3 grid, hipStream_t st, const TrialParams<Real>& p, bool* found,
                      hipFuncAttributes* a) {
  *found = true;
  switch (k.ch) {
    case CH_RAYLEIGH:
      return k.csi ? go<T, NSLOT, AL, CH_RAYLEIGH, true>(grid, st, p, a)
                   : go<T, NSLOT, AL, CH_RAYLEIGH, false>(grid, st, p, a);
    case CH_LOS:
      return k.csi ? go<T, NSLOT, AL, CH_LOS, true>(grid, st, p, a) : go<T, NSLOT, AL, CH_LOS, false>(grid, st, p, a);
    case CH_TWOPATH:
      return k.csi ? go<T, NSLOT, AL, CH_TWOPATH, true>(grid, st, p, a)
                   : go<T, NSLOT, AL, CH_TWOPATH, false>(grid, st, p, a);
    case CH_TABLE:
      return k.csi ? go<T, NSLOT, AL, CH_TABLE, true>(grid, st, p, a)
                   : go<T, NSLOT, AL, CH_TABLE, false>(grid, st, p, a);
    default:
      *found = false;
      return hipSuccess;
  }
}

template <int T>
hipError_t by_team(const InstanceKey& k, dim3 grid, hipStream_t st, const TrialParams<Real>& p, bool* found,
                   hipFuncAttributes* a) {
  constexpr int P = kF / T;
  if (k.aligned) {
    if constexpr (8 < P) {
      if (k.nslot == 8) return by_channel<T, 8, true>(k, grid, st, p, found, a);
    }
    if constexpr (4 < P) {
      if (k.nslot == 4) return by_channel<T, 4, true>(k, grid, st, p, found, a);
    }
    return hipSuccess;
  }
  if (k.nslot != P) return hipSuccess;
  return by_channel<T, P, false>(k, grid, st, p, found, a);
}

}  // namespace

#if INST_F64
#define MIMO_LAUNCH_NAME MIMO_CAT(MIMO_CAT(launch_trial_F, INST_F), _f64)
#else
#define MIMO_LAUNCH_NAME MIMO_CAT(MIMO_CAT(launch_trial_F, INST_F), _f32)
#endif
hipError_t MIMO_LAUNCH_NAME(const InstanceKey& k, dim3 grid, hipStream_t st, const TrialParams<Real>& p, bool* found,
                            hipFuncAttributes* attr) {
  *found = false;
  if (k.F != kF || k.f64 != kF64) return hipSuccess;
  if constexpr (kF64) {
    if (k.T == team_size64(kF)) return by_team<team_size64(kF)>(k, grid, st, p, found, attr);
  } else {
    if (k.T == team_size(kF)) return by_team<team_size(kF)>(k, grid, st, p, found, attr);
    if constexpr (alt_team_size(kF) != team_size(kF)) {
      if (k.T == alt_team_size(kF)) return by_team<alt_team_size(kF)>(k, grid, st, p, found, attr);
    }
  }
  return hipSuccess;
}

}  // namespace mimo
