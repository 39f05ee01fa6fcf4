#!/bin/bash
# Per-config rocprofv3 PMC passes behind bench.py's roofline (run on the GPU box):
#   c4  : the headline launch only (C4, 10M 17-clue puzzles, default solver), every other leg off
#   c3  : the checker launch only (100M boards), C4 shrunk to 1024 puzzles
#   cal : tools/fetch_calib (the solvers' byte-load / byte-store pattern, known byte counts)
# One counter group per rocprofv3 run (FETCH_SIZE and WRITE_SIZE cannot share a pass).
# usage: tools/pmc_c4.sh <outdir>     then: python3 tools/pmc_c4_summary.py <outdir>
set -o pipefail
out=$1; root=$(pwd); mkdir -p "$out"; export TMPDIR=/tmp
OFF="--c2-puzzles 0 --minimal-puzzles 0 --hard-leg 0 --count-leg 0 --lane-puzzles 0 --cpu-seconds 0 --http-requests 0 --pmc-summary="
C4="$root/bench.py --steps 2 --warmup 1 --check-boards 0 $OFF"
C3="$root/bench.py --steps 1 --warmup 0 --batch 1024 --check-boards 100000000 --check-steps 2 --check-warmup 1 $OFF"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
# stall attribution per wave-cycle (waiting on a counter / issue-stalled / issuing; LDS share)
SQW="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM"
run() {  # <tag> <counters> <program...>
  local tag=$1 ctr=$2; shift 2
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d "$root/$out/$tag" -o run -- "$@" \
     > "$root/$out/$tag.log" 2>&1) || { echo "pass $tag failed"; tail -5 "$out/$tag.log"; exit 1; }
  echo "pass $tag ok"
}
run cal_fetch FETCH_SIZE "$root/tools/fetch_calib" 10000000
run cal_write WRITE_SIZE "$root/tools/fetch_calib" 10000000
run c4_fetch FETCH_SIZE python3 $C4
run c4_write WRITE_SIZE python3 $C4
run c4_sq "$SQ" python3 $C4
run c4_sqw "$SQW" python3 $C4
run c3_fetch FETCH_SIZE python3 $C3
run c3_write WRITE_SIZE python3 $C3
run c3_sq "$SQ" python3 $C3
python3 tools/pmc_c4_summary.py "$out"
