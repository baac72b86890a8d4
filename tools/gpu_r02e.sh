# Round-2e check: full GPU suite (-rA -s), smoke, default bench line, the fp64 lines the
# fp64 pipeline / F = 8192 team change touches (paper F 4096, config-5 array F 8192).
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r02e}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA -s --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
cat $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_f64.json 2> $O/bench.err || exit $?
cat $O/bench_f64.json
timeout -k 10 300 python bench.py --workload paper --batch 32768 --steps 5 --no-cpu-baseline > $O/bench_paper.json 2>> $O/bench.err || exit $?
cat $O/bench_paper.json
timeout -k 10 300 python bench.py --workload 5su --batch 2048 --steps 5 --no-cpu-baseline > $O/bench_5su.json 2>> $O/bench.err || exit $?
cat $O/bench_5su.json
bash tools/gpu_ab2.sh $O/ab2k_f32_pipe -none- "abl/v2k_base.so abl/v2k_np32.so --rounds 6 --precision f32" || exit $?
timeout -k 10 300 python bench.py --workload 5su --batch 2048 --steps 5 --precision f32 --no-cpu-baseline > $O/bench_5su_f32.json 2>> $O/bench.err || exit $?
MIMO_TEAM=1024 timeout -k 10 300 python bench.py --workload 5su --batch 2048 --steps 5 --precision f32 --no-cpu-baseline > $O/bench_5su_f32_t1024.json 2>> $O/bench.err || exit $?
python -c "
import json
for f in ['bench_5su_f32','bench_5su_f32_t1024']:
    d=json.load(open('$O/'+f+'.json')); print(f, d['ms_per_step'], d['value'], d['roofline']['kernel'])"
