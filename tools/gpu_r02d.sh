set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_config4.py -m gpu -v -rA -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_ab2.sh $O/ab2k -none- "abl/lib_cur.so abl/lib_pf64.so abl/lib_nopipe.so abl/lib_pfnp.so --rounds 6 --precision f64" || exit $?
bash tools/gpu_ab2.sh $O/ab4k -none- "abl/lib_cur4k.so abl/lib_pf4k.so abl/lib_np4k.so abl/lib_pfnp4k.so --rounds 6 --precision f64 --workload paper --batch 32768"
