# Round 3 (session 3): stage-2 twiddle rows r = 3, 5, 6 from LDS (ltw2) and, on top, the
# wave-split inverse's w3 inter-step twiddle loaded instead of formed (ltw2_w3), against the
# session's HEAD (base2k); F 2048 variant builds, config 2 and CSI / LoS.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03x}
mkdir -p $O
show() { python -c "import json; [print('$1', round(d['median_ms'],3), round(d['min_ms'],3), d['errors'], d['lib']) for d in json.load(open('$O/$1.json'))]"; }
timeout -k 10 400 python tools/ab_libs.py abl/lib_base2k.so abl/lib_ltw2.so abl/lib_ltw2_w3.so --rounds 8 > $O/ab_2.json 2> $O/ab_2.err && show ab_2 || exit $?
timeout -k 10 300 python tools/ab_libs.py abl/lib_base2k.so abl/lib_ltw2.so abl/lib_ltw2_w3.so --rounds 4 --workload 2los > $O/ab_2los.json 2> $O/ab_2los.err && show ab_2los || exit $?
timeout -k 10 300 python tools/ab_libs.py abl/lib_base2k.so abl/lib_ltw2.so abl/lib_ltw2_w3.so --rounds 3 --batch 16384 --iters 0,1,2 --workload 2mcnc > $O/ab_2mcnc.json 2> $O/ab_2mcnc.err && show ab_2mcnc || exit $?
