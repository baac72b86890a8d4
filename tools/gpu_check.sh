set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -q -m gpu -s > gpurun_out/gpu3.log 2>&1 && echo TESTS_OK >> gpurun_out/gpu3.log
timeout -k 10 300 python bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1 -o run -- python3 bench.py --no-cpu-baseline --steps 5 > gpurun_out/prof1.log 2>&1
