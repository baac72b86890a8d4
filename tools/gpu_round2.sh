# Round-2 measurement call: full GPU suite (-rA -s kept), f64 headline bench + rocprof stats
# of the same command + FETCH/WRITE PMC passes, then secondary lines (f32, paper, CNC, MCNC,
# LoS, two-path, CSI, config-5 array) and the config-4 sweep.
# usage: bash tools/gpu_round2.sh <outdir> [skip-tests]
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/round2}
mkdir -p $O
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA -s --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
B="bench.py --steps 10 --warmup 2"
timeout -k 10 300 python $B > $O/bench_f64.json 2> $O/bench_f64.err || exit $?
cat $O/bench_f64.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $B --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_write.log 2>&1 || exit $?
timeout -k 10 300 python $B --precision f32 --no-cpu-baseline > $O/bench_f32.json 2> $O/bench_f32.err || exit $?
timeout -k 10 300 python bench.py --iters 0,1,2,3,4 --cpu-seconds 10 > $O/bench_cnc4.json 2> $O/bench_cnc4.err || exit $?
timeout -k 10 300 python bench.py --workload paper --batch 32768 --cpu-seconds 10 > $O/bench_paper.json 2> $O/bench_paper.err || exit $?
for w in 2los 2twopath 2csi; do timeout -k 10 300 python bench.py --workload $w --steps 5 --cpu-seconds 5 > $O/bench_$w.json 2> $O/bench_$w.err || exit $?; done
timeout -k 10 300 python bench.py --workload 2mcnc --iters 0,1,2 --batch 16384 --steps 3 --cpu-seconds 5 > $O/bench_2mcnc.json 2> $O/bench_2mcnc.err || exit $?
timeout -k 10 300 python bench.py --workload 5su --batch 2048 --steps 3 --cpu-seconds 10 > $O/bench_5su.json 2> $O/bench_5su.err || exit $?
timeout -k 10 300 python tools/fixed_ber_check.py --channel rayleigh --receiver cnc > $O/sweep_cnc_rayleigh.json 2> $O/sweep.err || exit $?
echo done > $O/done.txt
