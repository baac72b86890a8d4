# One GPU call: parity tests (both precisions), then short f64 / f32 bench lines.
# Usage: bash tools/gpu_step.sh "<pytest targets>" [bench args]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TESTS=${1:-tests}
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -v -rA -s --timeout 180 --timeout-method thread > gpurun_out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest.log | tail -3
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 --precision f64 > gpurun_out/bench_f64.json 2> gpurun_out/bench_f64.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 --precision f32 > gpurun_out/bench_f32.json 2> gpurun_out/bench_f32.err || exit $?
cat gpurun_out/bench_f64.json gpurun_out/bench_f32.json
exit $rc
