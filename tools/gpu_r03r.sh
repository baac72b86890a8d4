# Round 3 (session 2) PMC record of the shipped kernels: FETCH / WRITE traffic of config 2
# (the bench line's roofline.traffic) and one SQ pass each for config 2, the paper config
# and the config-5 array (VALU busy, waits, LDS conflicts).
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03r}
mkdir -p $O
B="bench.py --no-cpu-baseline --steps 2 --warmup 1"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c2_fetch -o run -- python3 $B > $O/c2_fetch.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c2_write -o run -- python3 $B > $O/c2_write.log 2>&1 || exit 1
python tools/pmc_traffic.py $O/c2_fetch $O/c2_write $O/pmc_traffic_f64.json --workload 2 --iters 0 --precision f64 --batch 65536 || exit 1
cat $O/pmc_traffic_f64.json
SQ="SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
for wl in "2 65536" "paper 32768" "5su 2048"; do
  set -- $wl
  timeout -k 10 240 rocprofv3 --pmc $SQ GRBM_GUI_ACTIVE --output-format csv -d $O/sq_$1 -o run -- python3 $B --workload $1 --batch $2 > $O/sq_$1.log 2>&1 || exit 1
  python tools/pmc_summary.py $O/sq_$1 > $O/sq_$1.txt || exit 1
  echo "== $1"; cat $O/sq_$1.txt
done
