# Round 3 (session 2): the fp64 cuts after gating the folded precode to the wave-split
# instances and keeping CSI at 3 teams per CU; old vs new Philox rounds at F 4096 / 8192.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03p}
mkdir -p $O
show() { python -c "import json; [print('$1', round(d['median_ms'],3), d['errors'], d['lib']) for d in json.load(open('$O/$1.json'))]"; }
timeout -k 10 400 python tools/ab_libs.py abl/lib_base4k.so abl/lib_x4k.so abl/lib_y4k.so --rounds 4 --batch 32768 --workload paper > $O/ab_paper.json 2> $O/ab_paper.err && show ab_paper || exit $?
timeout -k 10 600 python tools/ab_libs.py abl/lib_base8k.so abl/lib_x8k.so abl/lib_y8k.so --rounds 3 --batch 2048 --workload 5su > $O/ab_5su.json 2> $O/ab_5su.err && show ab_5su || exit $?
timeout -k 10 400 python tools/ab_libs.py abl/lib_base.so abl/lib_x2k.so --rounds 5 > $O/ab_2.json 2> $O/ab_2.err && show ab_2 || exit $?
timeout -k 10 400 python tools/ab_libs.py abl/lib_base.so abl/lib_x2k.so --rounds 3 --workload 2csi > $O/ab_2csi.json 2> $O/ab_2csi.err && show ab_2csi || exit $?
