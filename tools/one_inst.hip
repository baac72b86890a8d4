// Single-instance build for register / spill inspection:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -DXMW=3 -I<csrc> -c tools/one_inst.hip \
//         -Rpass-analysis=kernel-resource-usage      (fp64: -DXR=double -DXT=256 -DXNS=4 -DXMW=2)
#include "trial_kernel.h"
#ifndef XF
#define XF 2048
#endif
#ifndef XT
#define XT 128
#endif
#ifndef XNS
#define XNS 8
#endif
#ifndef XMW
#define XMW 3
#endif
#ifndef XCH
#define XCH 1
#endif
#ifndef XCSI
#define XCSI false
#endif
#ifndef XNB
#define XNB 1
#endif
#ifndef XR
#define XR float
#endif
#ifndef XSYM
#define XSYM (XNB == 1)
#endif
template __global__ void mimo::trial_kernel<XR, XF, XT, XNS, true, XCH, XCSI, XMW, XNB, XSYM>(mimo::TrialParams<XR>);
