# Round-3 secondary bench lines at HEAD (no CPU baseline except where noted): f32 config 2,
# CNC 0-4, paper config (+ CNC 0-8), LoS / two-path / CSI, MCNC, config-5 array f64 + f32.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03_lines}
mkdir -p $O
N="--no-cpu-baseline"
timeout -k 10 300 python bench.py --precision f32 $N > $O/bench_f32.json 2> $O/bench_f32.err || exit $?
timeout -k 10 300 python bench.py --iters 0,1,2,3,4 $N > $O/bench_cnc4.json 2> $O/bench_cnc4.err || exit $?
timeout -k 10 300 python bench.py --workload paper --batch 32768 $N > $O/bench_paper.json 2> $O/bench_paper.err || exit $?
timeout -k 10 300 python bench.py --workload paper --iters 0,1,2,3,4,5,6,7,8 --batch 32768 --steps 5 $N > $O/bench_paper_cnc8.json 2> $O/bench_paper_cnc8.err || exit $?
for w in 2los 2twopath 2csi; do timeout -k 10 300 python bench.py --workload $w --steps 5 $N > $O/bench_$w.json 2> $O/bench_$w.err || exit $?; done
timeout -k 10 300 python bench.py --workload 2mcnc --iters 0,1,2 --batch 16384 --steps 3 $N > $O/bench_2mcnc.json 2> $O/bench_2mcnc.err || exit $?
timeout -k 10 300 python bench.py --workload 5su --batch 2048 --steps 5 --cpu-seconds 10 > $O/bench_5su.json 2> $O/bench_5su.err || exit $?
timeout -k 10 300 python bench.py --workload 5su --batch 2048 --steps 5 --precision f32 $N > $O/bench_5su_f32.json 2> $O/bench_5su_f32.err || exit $?
for f in $O/bench_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f'.split('/')[-1], d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['dtype'])"; done
