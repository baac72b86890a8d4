# New GPU tests (multi-point, 16 workers, gloo sweep), config-4 published-grid checks, f64 A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_points.py tests/test_gpu_link.py -m gpu -x -v -rA -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for c in rayleigh los two_path; do
  timeout -k 10 300 python tools/fixed_ber_check.py --channel $c --receiver cnc --out $O/cnc_$c.npz > $O/cnc_$c.json 2>> $O/fb_err.log || exit $?
  cat $O/cnc_$c.json
done
timeout -k 10 300 python tools/fixed_ber_check.py --channel rayleigh --receiver mcnc --out $O/mcnc_rayleigh.npz > $O/mcnc_rayleigh.json 2>> $O/fb_err.log || exit $?
cat $O/mcnc_rayleigh.json
bash tools/gpu_ab2.sh $O/ab64 -none- "abl/lib_lut.so abl/lib_twall.so abl/lib_pf64.so abl/lib_nopipe.so abl/lib_maxilp.so --rounds 6 --precision f64"
