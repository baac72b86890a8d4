set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_points.py tests/test_gpu_link.py tests/test_gpu_config4.py -m gpu -v -rA -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --workload paper --iters 0,1,2,3,4,5,6,7,8 --batch 32768 --steps 5 --no-cpu-baseline > $O/bench_paper_cnc8.json 2> $O/bench_paper.err || exit $?
cat $O/bench_paper_cnc8.json
bash tools/gpu_ab2.sh $O/ab64 -none- "abl/lib_cur.so abl/lib_twall.so abl/lib_pf64.so abl/lib_nopipe.so abl/lib_maxilp.so --rounds 6 --precision f64"
