#!/bin/bash
# Round-3 rocprofv3 PMC passes behind bench.py's roofline and the stall attribution of the
# search kernel (run on the GPU box, one counter group per rocprofv3 run):
#   cal / calw : tools/fetch_calib with the solvers' byte pattern (mode 0) and with the same
#                records written 16 at a time by 16-B stores (mode 1): what WRITE_SIZE reports
#                for 81-B records written one by one
#   c4         : the headline launch (C4, 10M 17-clue puzzles), traffic + two SQ groups
#   c3         : the checker launch (100M boards)
#   min / hard : solve_profile.py on the minimal and hard workloads (plain kernel, no donation)
# usage: tools/pmc_r03.sh <outdir> [passes...]    then: python3 tools/pmc_c4_summary.py <outdir>
set -o pipefail
out=$1; shift; root=$(pwd); mkdir -p "$out"; export TMPDIR=/tmp
passes=${*:-cal calw c4 c3 min hard}
OFF="--c2-puzzles 0 --minimal-puzzles 0 --hard-leg 0 --count-leg 0 --lane-puzzles 0 --cpu-seconds 0 --http-requests 0 --pmc-summary="
C4="$root/bench.py --steps 2 --warmup 1 --check-boards 0 $OFF"
C3="$root/bench.py --steps 1 --warmup 0 --batch 1024 --check-boards 100000000 --check-steps 2 --check-warmup 1 $OFF"
MIN="$root/tools/solve_profile.py --workload minimal --n 1048576 --reps 2 --donate 0 --solver quad"
HARD="$root/tools/solve_profile.py --workload hard --n 100000 --reps 2 --donate 0 --solver quad"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
SQW="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM"
run() {  # <tag> <counters> <program...>
  local tag=$1 ctr=$2; shift 2
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d "$root/$out/$tag" -o run -- "$@" \
     > "$root/$out/$tag.log" 2>&1) || { echo "pass $tag failed"; tail -5 "$out/$tag.log"; exit 1; }
  echo "pass $tag ok"
}
for p in $passes; do
  case $p in
  cal)  run cal_fetch FETCH_SIZE "$root/tools/fetch_calib" 10000000 0
        run cal_write WRITE_SIZE "$root/tools/fetch_calib" 10000000 0 ;;
  calw) run calw_fetch FETCH_SIZE "$root/tools/fetch_calib" 10000000 1
        run calw_write WRITE_SIZE "$root/tools/fetch_calib" 10000000 1 ;;
  c4)   run c4_fetch FETCH_SIZE python3 $C4
        run c4_write WRITE_SIZE python3 $C4
        run c4_sq "$SQ" python3 $C4
        run c4_sqw "$SQW" python3 $C4 ;;
  c3)   run c3_fetch FETCH_SIZE python3 $C3
        run c3_write WRITE_SIZE python3 $C3
        run c3_sq "$SQ" python3 $C3 ;;
  min)  run min_sq "$SQ" python3 $MIN
        run min_sqw "$SQW" python3 $MIN ;;
  hard) run hard_sq "$SQ" python3 $HARD
        run hard_sqw "$SQW" python3 $HARD ;;
  *) echo "unknown pass $p"; exit 2 ;;
  esac
done
python3 tools/pmc_c4_summary.py "$out"
