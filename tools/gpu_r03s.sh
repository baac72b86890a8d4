# Round 3 (session 2): cold paths out of line (general-p Rapp, the exact alpha fallback):
# no hoisted constants spilled per trial.  base = session start, x/y = previous step, z = now.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03s}
mkdir -p $O
show() { python -c "import json; [print('$1', round(d['median_ms'],3), d['errors'], d['lib']) for d in json.load(open('$O/$1.json'))]"; }
timeout -k 10 400 python tools/ab_libs.py abl/lib_base.so abl/lib_x2k.so abl/lib_z2k.so --rounds 5 > $O/ab_2.json 2> $O/ab_2.err && show ab_2 || exit $?
for w in 2csi 2los 2twopath; do
  timeout -k 10 400 python tools/ab_libs.py abl/lib_base.so abl/lib_x2k.so abl/lib_z2k.so --rounds 3 --workload $w > $O/ab_$w.json 2> $O/ab_$w.err && show ab_$w || exit $?
done
timeout -k 10 400 python tools/ab_libs.py abl/lib_base.so abl/lib_x2k.so abl/lib_z2k.so --rounds 3 --batch 16384 --iters 0,1,2 --workload 2mcnc > $O/ab_2mcnc.json 2> $O/ab_2mcnc.err && show ab_2mcnc || exit $?
timeout -k 10 400 python tools/ab_libs.py abl/lib_base4k.so abl/lib_y4k.so abl/lib_z4k.so --rounds 4 --batch 32768 --workload paper > $O/ab_paper.json 2> $O/ab_paper.err && show ab_paper || exit $?
timeout -k 10 600 python tools/ab_libs.py abl/lib_base8k.so abl/lib_y8k.so abl/lib_z8k.so --rounds 3 --batch 2048 --workload 5su > $O/ab_5su.json 2> $O/ab_5su.err && show ab_5su || exit $?
