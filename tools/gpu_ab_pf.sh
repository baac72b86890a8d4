set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
# Interleaved A/B: twiddle prefetch at the start of each transform (and fewer loaded powers).
timeout -k 10 300 python tools/ab_libs.py abl/lib_dpp_2048.so abl/lib_pf_2048.so abl/lib_pf1_2048.so abl/lib_pf2_2048.so --rounds 8 > gpurun_out/ab_pf_2.json 2>&1 && \
timeout -k 10 300 python tools/ab_libs.py abl/lib_dpp_4096.so abl/lib_pf_4096.so --rounds 6 --batch 32768 --workload paper > gpurun_out/ab_pf_paper.json 2>&1 && \
timeout -k 10 300 python tools/ab_libs.py abl/lib_dpp_8192.so abl/lib_pf_8192.so --rounds 4 --batch 4096 --workload 5su > gpurun_out/ab_pf_5su.json 2>&1
rc=$?; echo "rc=$rc"; exit $rc
