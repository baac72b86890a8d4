# Round 3 (session 3) final check after the LDS stage-2 twiddles and the micro cuts: full GPU suite, smoke, headline bench + rocprof,
# and the F 2048 secondary lines.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03z}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rA -s --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
cat $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --steps 5 > $O/prof.log 2>&1 || exit $?
N="--no-cpu-baseline"
timeout -k 10 300 python bench.py --iters 0,1,2,3,4 $N > $O/bench_cnc4.json 2> $O/bench_cnc4.err || exit $?
for w in 2los 2twopath 2csi; do timeout -k 10 300 python bench.py --workload $w --steps 5 $N > $O/bench_$w.json 2> $O/bench_$w.err || exit $?; done
timeout -k 10 300 python bench.py --workload 2mcnc --iters 0,1,2 --batch 16384 --steps 3 $N > $O/bench_2mcnc.json 2> $O/bench_2mcnc.err || exit $?
for f in $O/bench*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f'.split('/')[-1], d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['dtype'])"; done

timeout -k 10 300 python bench.py --workload paper --batch 32768 $N > $O/bench_paper.json 2> $O/bench_paper.err || exit $?
timeout -k 10 300 python bench.py --workload paper --iters 0,1,2,3,4,5,6,7,8 --batch 32768 --steps 5 $N > $O/bench_paper_cnc8.json 2> $O/bench_paper_cnc8.err || exit $?
timeout -k 10 300 python bench.py --workload 5su --batch 2048 --steps 3 $N > $O/bench_5su.json 2> $O/bench_5su.err || exit $?
timeout -k 10 300 python tools/fixed_ber_check.py --grid baseline > $O/c4_baseline.json 2> $O/c4_baseline.err || exit $?
for f in $O/bench_paper*.json $O/bench_5su.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f'.split('/')[-1], d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['dtype'])"; done
cut -c1-400 $O/c4_baseline.json
true
B="bench.py --no-cpu-baseline --steps 2 --warmup 1"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c2_fetch -o run -- python3 $B > $O/c2_fetch.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c2_write -o run -- python3 $B > $O/c2_write.log 2>&1 || exit 1
python tools/pmc_traffic.py $O/c2_fetch $O/c2_write $O/pmc_traffic_f64.json --workload 2 --iters 0 --precision f64 --batch 65536 || exit 1
grep -E "hbm_bytes" $O/pmc_traffic_f64.json
B5="bench.py --no-cpu-baseline --steps 2 --warmup 1 --workload 5su --batch 2048"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c5_fetch -o run -- python3 $B5 > $O/c5_fetch.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c5_write -o run -- python3 $B5 > $O/c5_write.log 2>&1 || exit 1
python tools/pmc_traffic.py $O/c5_fetch $O/c5_write $O/pmc_traffic_5su.json --workload 5su --iters 0 --precision f64 --batch 2048 || exit 1
grep -E "hbm_bytes" $O/pmc_traffic_5su.json
exit $rc
