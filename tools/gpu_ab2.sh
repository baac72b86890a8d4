# GPU parity subset, then interleaved A/B of library builds (one process), optional microbench.
# usage: bash tools/gpu_ab2.sh <out-dir> "<pytest targets or -none->" "<ab_libs args>" ["<extra cmd>"]
set -o pipefail
export TMPDIR=/tmp
O=$1
mkdir -p $O
if [ -n "$4" ]; then timeout -k 10 120 bash -c "$4" > $O/extra.log 2>&1 || exit $?; fi
if [ "$2" != "-none-" ]; then
  timeout -k 10 600 python -u -m pytest $2 -m gpu -x -q -rA -s --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
timeout -k 10 600 python tools/ab_libs.py $3 > $O/ab.json 2> $O/ab.err || exit $?
python -c "
import json; d=json.load(open('$O/ab.json'))
for x in d: print(x['lib'], x['desc'], round(x['median_ms'],3), x['errors'])"
