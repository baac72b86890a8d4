# Ablation of the fused kernel (wrong results by design, timing only) + PMC passes.
# usage: bash tools/gpu_abl.sh <precision> <outdir>
set -o pipefail
export TMPDIR=/tmp
PREC=${1:-f64}
O=${2:-gpurun_out/abl}
mkdir -p $O
MIMO_LIB=m-mimo-ofdm-with-nonlinear-pa-sim_amd/libmimo_engine_ablation.so timeout -k 10 300 python tools/ab_bench.py --precision $PREC --rounds 4 \
  --var MIMO_ABLATE=0 --var MIMO_ABLATE=1 --var MIMO_ABLATE=2 --var MIMO_ABLATE=4 --var MIMO_ABLATE=8 --var MIMO_ABLATE=16 --var MIMO_ABLATE=3 \
  > $O/ablation_$PREC.json 2> $O/ablation_$PREC.err || exit $?
bash tools/gpu_pmc.sh $O/pmc_$PREC
