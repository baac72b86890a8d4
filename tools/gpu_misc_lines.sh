# Secondary lines at HEAD: config-5 array in f32, and the N>1 bench path rehearsed with
# 2 gloo ranks sharing the one GPU (MIMO_BENCH_BACKEND=gloo).
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/misc}
mkdir -p $O
timeout -k 10 300 python bench.py --workload 5su --batch 4096 --steps 5 --precision f32 --no-cpu-baseline > $O/bench_5su_f32.json 2> $O/bench_5su_f32.err || exit $?
cat $O/bench_5su_f32.json
MIMO_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 1 > $O/bench_w2_gloo.json 2> $O/bench_w2_gloo.err || exit $?
cat $O/bench_w2_gloo.json
