set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=m-mimo-ofdm-with-nonlinear-pa-sim_amd/libmimo_engine.so
timeout -k 10 300 python tools/ab_libs.py abl/lib_nocache_2048.so $L --rounds 5 > gpurun_out/ab_2.json 2>&1 && \
timeout -k 10 300 python tools/ab_libs.py abl/lib_nocache_2048.so $L --rounds 3 --batch 16384 --iters 0,1,2 --workload 2mcnc > gpurun_out/ab_2mcnc.json 2>&1 && \
timeout -k 10 300 python tools/ab_libs.py abl/lib_nocache_4096.so $L --rounds 4 --batch 32768 --workload paper > gpurun_out/ab_paper.json 2>&1
rc=$?; echo "rc=$rc"; exit $rc
