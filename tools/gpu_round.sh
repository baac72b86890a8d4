# Round check on one MI355X: headline bench, config-3 variant, other workloads, kernel trace, PMC.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 python bench.py --iters 0,1,2,3,4 --no-cpu-baseline > gpurun_out/bench_cnc4.json 2> gpurun_out/bench_cnc4.err && \
timeout -k 10 300 python bench.py --workload paper --batch 32768 --cpu-seconds 10 > gpurun_out/bench_paper.json 2> gpurun_out/bench_paper.err && \
timeout -k 10 300 python bench.py --workload 5su --batch 4096 --steps 5 --cpu-seconds 10 > gpurun_out/bench_5su.json 2> gpurun_out/bench_5su.err && \
for w in 2los 2twopath 2csi; do timeout -k 10 300 python bench.py --workload $w --steps 5 --cpu-seconds 5 > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || exit 1; done && \
timeout -k 10 300 python bench.py --workload 2mcnc --iters 0,1,2 --batch 16384 --steps 3 --cpu-seconds 5 > gpurun_out/bench_2mcnc.json 2> gpurun_out/bench_2mcnc.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline --steps 5 > gpurun_out/prof.log 2>&1 && \
bash tools/gpu_pmc.sh gpurun_out/pmc_round
rc=$?; echo "done rc=$rc" > gpurun_out/round_done.txt; exit $rc
