set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline --steps 5 > gpurun_out/prof.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; cat gpurun_out/bench.json; exit $rc
