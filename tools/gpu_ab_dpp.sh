set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
# GPU tests of the production library, then interleaved A/B of the DPP wave sums.
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python tools/ab_libs.py abl/lib_p1_2048.so abl/lib_dpp_2048.so --rounds 8 > gpurun_out/ab_dpp_2.json 2>&1 && \
timeout -k 10 300 python tools/ab_libs.py abl/lib_p1_4096.so abl/lib_dpp_4096.so --rounds 6 --batch 32768 --workload paper > gpurun_out/ab_dpp_paper.json 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; exit $rc
