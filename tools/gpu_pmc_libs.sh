# PMC passes (SQ issue / wait breakdown) of the fused trial kernel for several library builds.
# usage: bash tools/gpu_pmc_libs.sh <outdir> "<bench args>" lib1.so lib2.so ...
set -o pipefail
export TMPDIR=/tmp
OUT=$1; shift
BARGS=$1; shift
mkdir -p $OUT
for lib in "$@"; do
  name=$(basename $lib .so); mkdir -p $OUT/$name
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
             "SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    MIMO_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/$name/p$i -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 $BARGS > $OUT/$name/p$i.log 2>&1 || { echo "pass $name $i failed"; exit 1; }
  done
  echo "== $name"; python tools/pmc_summary.py $OUT/$name
done
