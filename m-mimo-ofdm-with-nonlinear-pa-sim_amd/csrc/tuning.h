// Build-time A/B switches of the fused trial kernel, in one place.
//
// Each switch selects between two implementations that give identical per-trial counts; the
// default is the one that measured faster in an interleaved A/B on one MI355X (tools/ab_libs.py;
// the records are under profiles/, DESIGN.md §3 has the tables).  Override one for an A/B build:
//   make -C csrc variant VOUT=../../abl/lib_x.so VF=4096 VFLAGS=-DMIMO_PRE_EW_4096=0
// (Diagnostic-only switches that change results -- MIMO_DIAG_LUT_SEQ in real.h, MIMO_DIAG_ROWS2
// in wave_fft.h, MIMO_ABLATION -- stay next to the code they alter.)
#pragma once

// ---- occupancy (trial_inst.hip profile_for)
// fp64 F <= 2048: waves / SIMD the register allocation targets.  3: 168 VGPRs, 3 teams / CU.
// 4 (with the exchange LDS halved, diagnostic) measured +3.1 %: 73 VGPRs spill
// (profiles/r06/w4/).
#ifndef MIMO_W64_2048
#define MIMO_W64_2048 3
#endif

// ---- the Bussgang gain alpha_a per antenna (trial_kernel.h array_pass)
// Formed by one wave per antenna and handed over in LDS (0: every wave forms it): config 2
// -1.0 %, CSI -1.2 %, config-5 array -2.3 % (profiles/r05/ab/ab_*_alpha1.json).
#ifndef MIMO_ALPHA1
#define MIMO_ALPHA1 1
#endif
// ... at F 4096 (fp64) too since round 6, with the cold paths out of line there: -1.4 % together
// (profiles/r06/k4096/; alone +0.8 % in round 5).
#ifndef MIMO_ALPHA1_4096
#define MIMO_ALPHA1_4096 1
#endif

// ---- Philox rounds whose words are uniform across the team on the SALU (philox.h kUni)
// Always in the fp64 wave-split instances (F <= 2048).  F 4096: with CSI only (-2.4 % on the
// paper-CSI line, +1.1 % without CSI, profiles/r06/k4096/).  F 8192: with the folded weight
// below (-1.6 % for both, profiles/r06/k8192/).
#ifndef MIMO_UNI_4096_CSI
#define MIMO_UNI_4096_CSI 1
#endif
#ifndef MIMO_UNI_8192
#define MIMO_UNI_8192 1
#endif

// ---- CSI pass 1 in polar form (Rayleigh CSI instances, fp64): -4.8 % on the CSI line
// (profiles/r05/ab/ab_2csi_polar.json).  0: two Cartesian Box-Muller draws per slot.
#ifndef MIMO_CSI_POLAR
#define MIMO_CSI_POLAR 1
#endif

// ---- the precoding weight w = 1 / ||Hhat|| / sqrt(F) folded into the channel (PRE_EW; with
// perfect CSI the loops then carry h w, WSC, and the Rayleigh draws take w in their radius,
// WSC_RAY).  Wave-split instances: -1.1 % (round 3).  F 4096: -2.8 % once the cold paths were out
// of line (round 6); F 8192: -1.3 %.  Not with CSI: +3.1 % at F 4096, the F 2048 CSI line -1.3 %
// without it (profiles/r06/k2048/ab_2csi_preew.json).
#ifndef MIMO_PRE_EW_4096
#define MIMO_PRE_EW_4096 1
#endif
#ifndef MIMO_PRE_EW_8192
#define MIMO_PRE_EW_8192 1
#endif
#ifndef MIMO_PRE_EW_CSI
#define MIMO_PRE_EW_CSI 0
#endif
#ifndef MIMO_WSC_RAY
#define MIMO_WSC_RAY 1
#endif

// ---- the cold paths (general-p Rapp, the exact-alpha fallback) out of line at F 4096 too:
// scratch 492 -> 288 B/lane, traffic 108 -> 31 KB per trial, paper -1.0 % (round 6; +1.6 % in
// round 3).  The other fp64 instances always have them out of line.
#ifndef MIMO_COLD_OUT_4096
#define MIMO_COLD_OUT_4096 1
#endif

// ---- |Hhat|^2 recomputed after the FFT (E2_RE) also with CSI: +1.7 % (F 2048) / +2.7 %
// (F 4096): the estimate stays live across both transforms (profiles/r06/k2048/ab_2csi_e2.json).
#ifndef MIMO_E2_RE_CSI
#define MIMO_E2_RE_CSI 0
#endif

// ---- F 4096: two int8 lattice levels per VGPR (SLAB8): -2.2 % in round 4; one level per word
// +3.9 % at round 6 (profiles/r06/k4096/ab_paper_s8.json).
#ifndef MIMO_SLAB8_4096
#define MIMO_SLAB8_4096 1
#endif

// ---- fp64 F 8192 (split_fft.h): two 4096-point sub-transforms on the lane halves and a
// radix-2 stage through v_permlane32_swap: -6.2 % against the 8192-point team (0: the team);
// their stages in cot-tan form: -2.4 % (profiles/r05/split/ab_5su_split.json).
#ifndef MIMO_SPLIT_FFT
#define MIMO_SPLIT_FFT 1
#endif
#ifndef MIMO_SPLIT_CT
#define MIMO_SPLIT_CT 1
#endif

// ---- team FFT (team_fft.h): the cot-tan constants of stage s + 1 loaded before stage s's
// exchange: paper +1.6 %, config-5 array +5.3 % (profiles/r06/k4096/, k8192/ab_5su_ctpf.json).
#ifndef MIMO_CT_PF
#define MIMO_CT_PF 0
#endif
