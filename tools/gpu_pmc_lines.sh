# FETCH_SIZE / WRITE_SIZE passes (separate runs) + kernel-trace stats for secondary bench lines.
# usage: bash tools/gpu_pmc_lines.sh <outdir>
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/pmc_lines}
mkdir -p $O
for wl in "5su 2048" "paper 32768"; do
  set -- $wl
  B="bench.py --no-cpu-baseline --steps 2 --warmup 1 --workload $1 --batch $2"
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${1}_fetch -o run -- python3 $B > $O/${1}_fetch.log 2>&1 || exit 1
  timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${1}_write -o run -- python3 $B > $O/${1}_write.log 2>&1 || exit 1
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${1}_stats -o run -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 --workload $1 --batch $2 > $O/${1}_bench.json 2> $O/${1}_stats.log || exit 1
  python tools/pmc_traffic.py $O/${1}_fetch $O/${1}_write $O/pmc_traffic_${1}.json --workload $1 --iters 0 --precision f64 --batch $2 || exit 1
  cat $O/pmc_traffic_${1}.json
done
