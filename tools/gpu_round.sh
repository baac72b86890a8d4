# Round check on one MI355X: headline bench, config-3 variant, kernel trace (tests run separately).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 python bench.py --iters 0,1,2,3,4 --no-cpu-baseline > gpurun_out/bench_cnc4.json 2> gpurun_out/bench_cnc4.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline --steps 5 > gpurun_out/prof.log 2>&1
rc=$?; echo "done rc=$rc" > gpurun_out/round_done.txt; exit $rc
