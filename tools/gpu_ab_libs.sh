# Interleaved A/B of library builds on one workload: bash tools/gpu_ab.sh <out> <workload> <batch> <rounds> lib...
set -o pipefail
export TMPDIR=/tmp
O=$1; W=$2; B=$3; R=$4; shift 4
mkdir -p $O
timeout -k 10 600 python tools/ab_libs.py "$@" --workload $W --batch $B --rounds $R > $O/ab_$W.json 2> $O/ab_$W.err || exit $?
python -c "import json; [print('$W', round(d['median_ms'],2), d['errors'], d['lib']) for d in json.load(open('$O/ab_$W.json'))]"
