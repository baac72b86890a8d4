set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_libs.py abl/lib_cur.so m-mimo-ofdm-with-nonlinear-pa-sim_amd/libmimo_engine.so abl/lib_pad5_8k.so --workload 5su --batch 4096 --rounds 3 > gpurun_out/ab3.json 2> gpurun_out/ab3.err
