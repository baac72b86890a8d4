# Round-2 closing measurement at HEAD: every bench line + rocprof + PMC (tools/gpu_round2.sh),
# the paper line at CNC 0-8 (config-4 comparison) and the config-5 array PMC after the diet.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r02g}
bash tools/gpu_round2.sh $O skip-tests || exit $?
timeout -k 10 300 python bench.py --workload paper --iters 0,1,2,3,4,5,6,7,8 --batch 32768 --steps 5 --no-cpu-baseline > $O/bench_paper_cnc8.json 2> $O/bench_paper_cnc8.err || exit $?
B="bench.py --no-cpu-baseline --steps 2 --warmup 1 --workload 5su --batch 2048"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/5su_fetch -o run -- python3 $B > $O/5su_fetch.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/5su_write -o run -- python3 $B > $O/5su_write.log 2>&1 || exit 1
python tools/pmc_traffic.py $O/5su_fetch $O/5su_write $O/pmc_traffic_5su.json --workload 5su --iters 0 --precision f64 --batch 2048 || exit 1
python tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/pmc_traffic_f64.json --workload 2 --iters 0 --precision f64 --batch 65536 || exit 1
