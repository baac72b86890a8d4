# Round 3, first GPU check after the knob cleanup + ADVICE fixes: full GPU suite, smoke,
# default bench line, the config-5 array line, rocprof stats of the default bench.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03f}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rA -s --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
cat $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
timeout -k 10 300 python bench.py --workload 5su --batch 2048 --steps 3 --no-cpu-baseline > $O/bench_5su.json 2> $O/bench_5su.err || exit $?
cat $O/bench_5su.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --steps 5 > $O/prof.log 2>&1 || exit $?
exit $rc
