# Round 3 (session 2): radix-16 DFT with the W8-type twiddles folded into FMAs (d) against
# the previous F 4096 / 8192 builds (y: before the cold-path change, z: after).
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03u}
mkdir -p $O
show() { python -c "import json; [print('$1', round(d['median_ms'],3), d['errors'], d['lib']) for d in json.load(open('$O/$1.json'))]"; }
timeout -k 10 400 python tools/ab_libs.py abl/lib_base4k.so abl/lib_y4k.so abl/lib_d4k.so --rounds 4 --batch 32768 --workload paper > $O/ab_paper.json 2> $O/ab_paper.err && show ab_paper || exit $?
timeout -k 10 600 python tools/ab_libs.py abl/lib_base8k.so abl/lib_z8k.so abl/lib_d8k.so --rounds 3 --batch 2048 --workload 5su > $O/ab_5su.json 2> $O/ab_5su.err && show ab_5su || exit $?
