set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
# Interleaved A/B: next antenna's channel draws inside the FFT exchange windows (MIMO_HPIPE).
timeout -k 10 300 python tools/ab_libs.py abl/lib_hp0_2048.so abl/lib_hp1_2048.so --rounds 8 > gpurun_out/ab_hp_2.json 2>&1 && \
timeout -k 10 300 python tools/ab_libs.py abl/lib_hp0_2048.so abl/lib_hp1_2048.so --rounds 3 --batch 16384 --iters 0,1,2 --workload 2mcnc > gpurun_out/ab_hp_2mcnc.json 2>&1 && \
timeout -k 10 300 python tools/ab_libs.py abl/lib_hp0_4096.so abl/lib_hp1_4096.so --rounds 6 --batch 32768 --workload paper > gpurun_out/ab_hp_paper.json 2>&1 && \
timeout -k 10 300 python tools/ab_libs.py abl/lib_hp0_8192.so abl/lib_hp1_8192.so --rounds 4 --batch 4096 --workload 5su > gpurun_out/ab_hp_5su.json 2>&1
rc=$?; echo "rc=$rc"; exit $rc
