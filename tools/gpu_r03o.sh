# Round 3 (session 2): which of the fp64 instruction cuts cost time at F 4096 / CSI?
# n = all cuts; h = Horner by plain fma (v_fmac + v_mov); p = old Philox; c = old precode.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03o}
mkdir -p $O
show() { python -c "import json; [print('$1', round(d['median_ms'],3), d['errors'], d['lib']) for d in json.load(open('$O/$1.json'))]"; }
timeout -k 10 400 python tools/ab_libs.py abl/lib_base4k.so abl/lib_n4k.so abl/lib_h4k.so abl/lib_p4k.so abl/lib_c4k.so --rounds 3 --batch 32768 --workload paper > $O/ab_paper.json 2> $O/ab_paper.err && show ab_paper || exit $?
timeout -k 10 400 python tools/ab_libs.py abl/lib_base.so abl/lib_n2k.so abl/lib_h2k.so abl/lib_p2k.so abl/lib_c2k.so --rounds 4 > $O/ab_2.json 2> $O/ab_2.err && show ab_2 || exit $?
timeout -k 10 400 python tools/ab_libs.py abl/lib_base.so abl/lib_n2k.so abl/lib_h2k.so abl/lib_p2k.so abl/lib_c2k.so --rounds 3 --workload 2csi > $O/ab_2csi.json 2> $O/ab_2csi.err && show ab_2csi || exit $?
