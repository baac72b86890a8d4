# Round 3 (session 2): interleaved A/B of the fp64 instruction cuts (HEAD build vs working
# tree, one-size variant libraries) on config 2 and its channel / receiver variants, the
# paper config (F 4096) and the config-5 array (F 8192); then the full GPU suite.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03n}
mkdir -p $O
A="abl/lib_base.so abl/lib_new.so"
show() { python -c "import json; [print('$1', round(d['median_ms'],3), d['errors'], d['lib']) for d in json.load(open('$O/$1.json'))]"; }
timeout -k 10 300 python tools/ab_libs.py $A --rounds 6 > $O/ab_2.json 2> $O/ab_2.err && show ab_2 || exit $?
for w in 2csi 2los 2twopath; do
  timeout -k 10 300 python tools/ab_libs.py $A --rounds 3 --workload $w > $O/ab_$w.json 2> $O/ab_$w.err && show ab_$w || exit $?
done
timeout -k 10 300 python tools/ab_libs.py $A --rounds 3 --iters 0,1,2,3,4 > $O/ab_cnc4.json 2> $O/ab_cnc4.err && show ab_cnc4 || exit $?
timeout -k 10 300 python tools/ab_libs.py abl/lib_base4k.so abl/lib_new4k.so --rounds 4 --batch 32768 --workload paper > $O/ab_paper.json 2> $O/ab_paper.err && show ab_paper || exit $?
timeout -k 10 600 python tools/ab_libs.py abl/lib_base8k.so abl/lib_new8k.so --rounds 4 --batch 2048 --workload 5su > $O/ab_5su.json 2> $O/ab_5su.err && show ab_5su || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; exit $rc
