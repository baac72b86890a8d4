# Round 3: HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the shipped fp64
# kernels at config 2 and the config-5 array, plus rocprof kernel stats of the 5su line.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03g}
mkdir -p $O
B2="bench.py --no-cpu-baseline --steps 2 --warmup 1"
B5="bench.py --no-cpu-baseline --steps 2 --warmup 1 --workload 5su --batch 2048"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f2 -o run -- python3 $B2 > $O/f2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w2 -o run -- python3 $B2 > $O/w2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f5 -o run -- python3 $B5 > $O/f5.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w5 -o run -- python3 $B5 > $O/w5.log 2>&1 || exit 1
python tools/pmc_traffic.py $O/f2 $O/w2 $O/pmc_traffic_f64.json --workload 2 --iters 0 --precision f64 --batch 65536 || exit 1
python tools/pmc_traffic.py $O/f5 $O/w5 $O/pmc_traffic_5su.json --workload 5su --iters 0 --precision f64 --batch 2048 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof5 -o run -- python3 bench.py --no-cpu-baseline --steps 5 --workload 5su --batch 2048 > $O/prof5.log 2>&1 || exit 1
cat $O/pmc_traffic_f64.json $O/pmc_traffic_5su.json
