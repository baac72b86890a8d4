set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
# GPU tests of the production library, then interleaved A/B of FFT plan / PA specialisation builds.
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python tools/ab_libs.py abl/lib_p0_2048.so abl/lib_p1_2048.so abl/lib_p1pas_2048.so --rounds 6 > gpurun_out/ab_plan_2.json 2>&1 && \
timeout -k 10 300 python tools/ab_libs.py abl/lib_p0_8192.so abl/lib_p1_8192.so abl/lib_p1pas_8192.so --rounds 4 --batch 4096 --workload 5su > gpurun_out/ab_plan_5su.json 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; cat gpurun_out/bench.json; exit $rc
