# Round-2f check after the F 8192 fp64 register diet: GPU suite, smoke, config-2 and config-5-array lines.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r02f}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA -s --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
cat $O/smoke.log
timeout -k 10 300 python bench.py --workload 5su --batch 2048 --steps 5 --no-cpu-baseline > $O/bench_5su.json 2>> $O/bench.err || exit $?
cat $O/bench_5su.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > $O/bench_f64_prof.json 2> $O/stats.log || exit $?
cat $O/bench_f64_prof.json
