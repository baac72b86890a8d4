# Round 3 (session 3): F 4096 cold paths split -- c4k0: both inline (shipped), c4k1: exact-alpha
# fallback out of line, c4k2: general-p Rapp out of line (paper config, 32,768 trials).
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03c4k}
mkdir -p $O
show() { python -c "import json; [print('$1', round(d['median_ms'],3), round(d['min_ms'],3), d['errors'], d['lib']) for d in json.load(open('$O/$1.json'))]"; }
timeout -k 10 500 python tools/ab_libs.py abl/lib_c4k0.so abl/lib_c4k1.so abl/lib_c4k2.so --rounds 6 --batch 32768 --workload paper > $O/ab_paper.json 2> $O/ab_paper.err && show ab_paper || exit $?
