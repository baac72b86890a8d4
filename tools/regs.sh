#!/bin/bash
# usage: tools/regs.sh [-DXMW=3 ...]  -> VGPRs / spills / occupancy of one trial_kernel instance
here=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -I"$here/m-mimo-ofdm-with-nonlinear-pa-sim_amd/csrc" \
  "$@" -c "$here/tools/one_inst.hip" -o /tmp/one_inst.o -Rpass-analysis=kernel-resource-usage 2>&1 \
  | grep -E "VGPRs:|AGPRs:|Spill|Occupancy|ScratchSize" | sed 's/.*remark: *//; s/ \[-Rpass.*//' | tr '\n' ' '; echo
