# The one GPU-box run script (replaces the per-session tools/gpu_r0*.sh / gpu_ab*.sh; their
# results stay under profiles/ and in git history).  Every GPU step has its own time limit and
# the steps are chained: the first failure ends the call.
#
#   bash tools/gpu.sh check <out>                      GPU suite (-rA -s), smoke, headline bench +
#                                                      rocprof stats, the secondary bench lines,
#                                                      config-4 grid at BASELINE extent
#   bash tools/gpu.sh lines <out> [workload ...]       bench lines only (default: every workload)
#   bash tools/gpu.sh ab <out> <name> "<ab_libs args>" lib.so ...
#                                                      interleaved A/B (tools/ab_libs.py)
#   bash tools/gpu.sh sq <out> "<bench args>" lib.so ...
#                                                      SQ issue / wait / LDS counter passes per library
#   bash tools/gpu.sh traffic <out> <name> "<bench args>"
#                                                      FETCH_SIZE / WRITE_SIZE passes -> pmc_traffic.json
#   bash tools/gpu.sh test <out> [pytest args]         the GPU suite (or a selection of it)
#   bash tools/gpu.sh c4 <out> [fixed_ber_check args]  config-4 grids (tools/fixed_ber_check.py)
#   bash tools/gpu.sh families <out> [family]          published CSI / BER-vs-IBO / small-array curves
#                                                      (tools/published_families.py)
#   bash tools/gpu.sh pairs <out>                      three-cornered hat over published re-runs
set -o pipefail
export TMPDIR=/tmp
MODE=$1; O=$2; shift 2
mkdir -p "$O"
N="--no-cpu-baseline --no-grid"  # bench lines and counter passes: the headline kernel only

line() {  # line <name> <bench args...>
  local name=$1; shift
  timeout -k 10 300 python bench.py $N "$@" > "$O/bench_$name.json" 2> "$O/bench_$name.err" || return $?
  python -c "import json; d=json.load(open('$O/bench_$name.json')); r=d['roofline']; print('$name', d['value'], r['kernel_ms'], round(r['frac'], 4), d['dtype'])"
}

lines() {
  local ws=("$@")
  [ ${#ws[@]} -eq 0 ] && ws=(2 cnc4 2los 2twopath 2csi 2mcnc paper paper_cnc8 papercsi 5su f32)
  for w in "${ws[@]}"; do
    case $w in
      2) line 2 --steps 5 || return $? ;;
      cnc4) line cnc4 --iters 0,1,2,3,4 --steps 5 || return $? ;;
      2mcnc) line 2mcnc --workload 2mcnc --iters 0,1,2 --batch 16384 --steps 3 || return $? ;;
      paper) line paper --workload paper --batch 32768 --steps 5 || return $? ;;
      paper_cnc8) line paper_cnc8 --workload paper --iters 0,1,2,3,4,5,6,7,8 --batch 32768 --steps 5 || return $? ;;
      papercsi) line papercsi --workload papercsi --batch 32768 --steps 5 || return $? ;;
      5su) line 5su --workload 5su --batch 2048 --steps 3 || return $? ;;
      f32) line f32 --precision f32 --steps 5 || return $? ;;
      *) line $w --workload $w --steps 5 || return $? ;;
    esac
  done
}

case $MODE in
  test)
    timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rA -s --timeout 300 --timeout-method thread "$@" > "$O/pytest_gpu.log" 2>&1
    rc=$?; tail -3 "$O/pytest_gpu.log"; exit $rc ;;
  check)
    timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rA -s --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
    rc=$?; echo "pytest rc=$rc"; tail -3 "$O/pytest_gpu.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit $?
    cat "$O/smoke.log"
    timeout -k 10 300 python bench.py > "$O/bench.json" 2> "$O/bench.err" || exit $?
    cat "$O/bench.json"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py $N --steps 5 > "$O/prof.log" 2>&1 || exit $?
    cp "$O"/prof/*/run_kernel_stats.csv "$O/bench_kernel_stats.csv" 2> /dev/null || cp "$O"/prof/run_kernel_stats.csv "$O/bench_kernel_stats.csv" 2> /dev/null
    lines || exit $?
    timeout -k 10 300 python tools/fixed_ber_check.py --grid baseline > "$O/c4_baseline.json" 2> "$O/c4_baseline.err" || exit $?
    cut -c1-300 "$O/c4_baseline.json"
    exit $rc ;;
  lines)
    lines "$@"; exit $? ;;
  ab)
    name=$1; args=$2; shift 2
    timeout -k 10 600 python tools/ab_libs.py "$@" $args > "$O/ab_$name.json" 2> "$O/ab_$name.err" || exit $?
    python -c "import json; [print('$name', round(d['median_ms'],3), round(d['min_ms'],3), d['errors'], d['lib']) for d in json.load(open('$O/ab_$name.json'))]" ;;
  sq)
    bargs=$1; shift
    for lib in "$@"; do
      name=$(basename "$lib" .so); mkdir -p "$O/$name"; i=0
      for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM" \
                 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
                 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 GRBM_GUI_ACTIVE"; do
        i=$((i+1))
        MIMO_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$O/$name/p$i" -o run -- python3 bench.py $N --steps 2 --warmup 1 $bargs > "$O/$name/p$i.log" 2>&1 || { echo "pass $name $i failed"; exit 1; }
      done
      echo "== $name"; python tools/pmc_summary.py "$O/$name" | tee "$O/$name/summary.txt"
    done ;;
  traffic)
    name=$1; bargs=$2
    B="bench.py $N --steps 2 --warmup 1 $bargs"
    timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/${name}_fetch" -o run -- python3 $B > "$O/${name}_fetch.log" 2>&1 || exit 1
    timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/${name}_write" -o run -- python3 $B > "$O/${name}_write.log" 2>&1 || exit 1
    python tools/pmc_traffic.py "$O/${name}_fetch" "$O/${name}_write" "$O/pmc_traffic_$name.json" $3 || exit 1
    grep -E "hbm_bytes" "$O/pmc_traffic_$name.json" ;;
  c4)
    timeout -k 10 600 python tools/fixed_ber_check.py "$@" > "$O/c4.json" 2> "$O/c4.err" || exit $?
    cut -c1-400 "$O/c4.json" ;;
  families)
    fam=${1:-all}
    timeout -k 10 900 python -u tools/published_families.py --family $fam --out "$O/families_$fam.json" > "$O/families_$fam.log" 2> "$O/families_$fam.err" || exit $?
    python -c "import json; [print(d['curve'], d['compared'], d['frac_abs_z_le1'], d['mean_z2'], d['max_abs_z'], d['median_abs_rel'], d['min_p_zero'], d['layout'], {k: v['mean_z2'] for k, v in d.items() if k.startswith('alt_')}) for d in json.load(open('$O/families_$fam.json'))]" ;;
  pairs)  # the three-cornered hat over the published re-run pairs + the calibrated csi1 curves
    timeout -k 10 900 python -u tools/published_families.py --pairs --out "$O/pairs.json" > "$O/pairs.log" 2> "$O/pairs.err" || exit $? ;;
  hat)    # the N-cornered hat over the BER-vs-IBO re-run groups
    timeout -k 10 900 python -u tools/published_families.py --hat --out "$O/hat.json" > "$O/hat.log" 2> "$O/hat.err" || exit $? ;;
  *)
    echo "unknown mode $MODE"; exit 2 ;;
esac
