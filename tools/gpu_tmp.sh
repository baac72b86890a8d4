set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -x -m gpu > gpurun_out/ab_tests.log 2>&1 && \
timeout -k 10 300 python tools/ab_libs.py abl/lib_prev.so m-mimo-ofdm-with-nonlinear-pa-sim_amd/libmimo_engine.so --rounds 6 > gpurun_out/ab1.json 2> gpurun_out/ab1.err
