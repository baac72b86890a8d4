set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_libs.py abl/lib_prev.so m-mimo-ofdm-with-nonlinear-pa-sim_amd/libmimo_engine.so abl/lib_nopoly4k.so --workload paper --batch 32768 --rounds 4 > gpurun_out/ab1.json 2> gpurun_out/ab1.err && \
timeout -k 10 300 python tools/ab_libs.py abl/lib_prev.so m-mimo-ofdm-with-nonlinear-pa-sim_amd/libmimo_engine.so --workload 5su --batch 4096 --rounds 4 > gpurun_out/ab2.json 2> gpurun_out/ab2.err
