set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_link.py -q -x -m gpu -k curve -s > gpurun_out/curve.log 2>&1
