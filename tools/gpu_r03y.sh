# Round 3 (session 3): micro cuts at F 2048 (the thread-0 pair swap on the Philox words,
# 4 selects instead of 8; the DC-hole scatter as 0/1 multiplies) against HEAD (ltw2h).
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03y}
mkdir -p $O
show() { python -c "import json; [print('$1', round(d['median_ms'],3), round(d['min_ms'],3), d['errors'], d['lib']) for d in json.load(open('$O/$1.json'))]"; }
timeout -k 10 400 python tools/ab_libs.py abl/lib_ltw2h.so abl/lib_micro.so --rounds 10 > $O/ab_2.json 2> $O/ab_2.err && show ab_2 || exit $?
timeout -k 10 300 python tools/ab_libs.py abl/lib_ltw2h.so abl/lib_micro.so --rounds 5 --workload 2csi > $O/ab_2csi.json 2> $O/ab_2csi.err && show ab_2csi || exit $?
timeout -k 10 300 python tools/ab_libs.py abl/lib_ltw2h.so abl/lib_micro.so --rounds 5 --workload 2los > $O/ab_2los.json 2> $O/ab_2los.err && show ab_2los || exit $?
timeout -k 10 300 python tools/ab_libs.py abl/lib_ltw2h.so abl/lib_micro.so --rounds 3 --batch 16384 --iters 0,1,2 --workload 2mcnc > $O/ab_2mcnc.json 2> $O/ab_2mcnc.err && show ab_2mcnc || exit $?
