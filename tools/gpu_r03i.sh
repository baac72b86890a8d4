# PMC of the shipped config-2 fp64 kernel (3 waves/SIMD): SQ issue/wait breakdown + HBM traffic.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03i}
mkdir -p $O
B2="bench.py --no-cpu-baseline --steps 2 --warmup 1"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f2 -o run -- python3 $B2 > $O/f2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w2 -o run -- python3 $B2 > $O/w2.log 2>&1 || exit 1
python tools/pmc_traffic.py $O/f2 $O/w2 $O/pmc_traffic_f64.json --workload 2 --iters 0 --precision f64 --batch 65536 || exit 1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/sq/p$i -o run -- python3 $B2 > $O/sq_p$i.log 2>&1 || exit 1
done
python tools/pmc_summary.py $O/sq > $O/sq_summary.txt
cat $O/pmc_traffic_f64.json $O/sq_summary.txt
