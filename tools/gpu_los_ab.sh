set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/los
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_config4.py tests/test_gpu_link.py -k "los or two_path or twopath or published" -m gpu -q -rA -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for w in 2los 2twopath; do timeout -k 10 300 python tools/ab_libs.py abl/lib_base.so abl/lib_los.so --rounds 6 --precision f64 --workload $w > $O/ab_$w.json 2> $O/ab_$w.err || exit $?; done
python -c "
import json
for w in ['2los','2twopath']:
    for x in json.load(open('$O/ab_'+w+'.json')): print(w, x['lib'], round(x['median_ms'],3), x['errors'])"
