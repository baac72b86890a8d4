# Round 3 (session 3): folded radix-16 DFT (W16^2 / W16^6 as c u with c in the column
# DFT-4's FMAs): GPU parity suite on the new library, then interleaved A/Bs against the
# HEAD library (abl/lib_head.so) at F 2048 (config 2), F 4096 (paper) and F 8192 (5su).
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03v}
mkdir -p $O
L=m-mimo-ofdm-with-nonlinear-pa-sim_amd/libmimo_engine.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
show() { python -c "import json; [print('$1', round(d['median_ms'],3), d['errors'], d['lib']) for d in json.load(open('$O/$1.json'))]"; }
timeout -k 10 300 python tools/ab_libs.py abl/lib_head.so $L --rounds 6 > $O/ab_2.json 2> $O/ab_2.err && show ab_2 || exit $?
timeout -k 10 300 python tools/ab_libs.py abl/lib_head.so $L --rounds 5 --batch 32768 --workload paper > $O/ab_paper.json 2> $O/ab_paper.err && show ab_paper || exit $?
timeout -k 10 400 python tools/ab_libs.py abl/lib_head.so $L --rounds 4 --batch 2048 --workload 5su > $O/ab_5su.json 2> $O/ab_5su.err && show ab_5su || exit $?
timeout -k 10 300 python tools/ab_libs.py abl/lib_head.so $L --rounds 4 --workload 2csi > $O/ab_2csi.json 2> $O/ab_2csi.err && show ab_2csi || exit $?
