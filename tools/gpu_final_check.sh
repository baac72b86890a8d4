# Full GPU suite (-rA -s kept) + smoke() + default bench line, as the driver runs them.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/final}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA -s --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
cat $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
exit $rc
