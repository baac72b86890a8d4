# Interleaved A/B of F 8192 fp64 builds on the config-5 array workload (5su).
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/ab8k}; shift
mkdir -p $O
timeout -k 10 600 python tools/ab_libs.py "$@" --workload 5su --batch 2048 --rounds 4 > $O/ab.json 2> $O/ab.err || exit $?
python -c "import json; [print(round(d['median_ms'],2), d['errors'], d['lib']) for d in json.load(open('$O/ab.json'))]"
