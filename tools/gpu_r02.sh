# Round-2 measurement call: GPU parity suite (kept with -rA -s), the f64 headline bench line,
# the rocprof kernel stats of the same bench command, FETCH/WRITE PMC passes, the f32 line.
# usage: bash tools/gpu_r02.sh [skip-tests]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02
mkdir -p $O
if [ "$1" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v -rA -s --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1
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
cat $O/bench_f32.json
echo done > $O/done.txt
