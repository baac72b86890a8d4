set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
# Interleaved A/B: FFT plan 1 with / without PA-specialised instances, max-ILP vs default scheduler.
timeout -k 10 400 python tools/ab_libs.py abl/lib_p1_2048.so abl/lib_p1_def_2048.so abl/lib_p1pas_2048.so \
  abl/lib_pas_def_2048.so abl/lib_pas_sb_2048.so abl/lib_pas_sbdef_2048.so --rounds 6 > gpurun_out/ab_sched_2.json 2>&1
rc=$?; echo "rc=$rc"; exit $rc
