# Round 3 (session 2): interleaved A/B of the fp64 F 2048 instruction cuts (HEAD build vs
# working tree, F 2048-only variant libraries), then the full GPU suite on the new library.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03m}
mkdir -p $O
A="abl/lib_base.so abl/lib_new.so"
timeout -k 10 300 python tools/ab_libs.py $A --rounds 6 > $O/ab_2.json 2> $O/ab_2.err || exit $?
cat $O/ab_2.json | grep -E '"(lib|median_ms|errors)"' 
timeout -k 10 300 python tools/ab_libs.py $A --rounds 3 --batch 16384 --iters 0,1,2 --workload 2mcnc > $O/ab_2mcnc.json 2> $O/ab_2mcnc.err || exit $?
timeout -k 10 300 python tools/ab_libs.py $A --rounds 3 --workload 2csi > $O/ab_2csi.json 2> $O/ab_2csi.err || exit $?
grep -hE '"(median_ms|errors)"' $O/ab_2mcnc.json $O/ab_2csi.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; exit $rc
