# Second PMC round: instruction fetch / cache, VMEM & LDS activity of the trial kernel.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc2
mkdir -p $OUT
BENCH="bench.py --no-cpu-baseline --steps 2 --warmup 1 --batch 16384"
i=0
for grp in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ" \
           "SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC" \
           "SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_SALU SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_UNALIGNED_STALL" \
           "SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_VALU_IOPS SQ_WAVES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $BENCH > $OUT/p$i.log 2>&1 || echo "pass $i failed" >> $OUT/failed.txt
done
