# F 8192 fp64: pair-wave FFT + block state memory -- parity, then interleaved A/B vs HEAD~ build.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03b}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sizes.py -k "8192 or config5" -v -rA -s --timeout 300 --timeout-method thread > $O/pytest_8k.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_8k.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/ab_libs.py abl/lib_base8k.so m-mimo-ofdm-with-nonlinear-pa-sim_amd/libmimo_engine.so --workload 5su --batch 2048 --rounds 4 > $O/ab_5su.json 2> $O/ab_5su.err || exit $?
cat $O/ab_5su.json
