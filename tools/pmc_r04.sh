#!/bin/bash
# Round-4 rocprofv3 PMC passes: what bounds solve4_kernel per SIMD.
# Counters per SIMD-cycle instead of summed per-wave activity, and the effective clock:
#   pipe : SQ_CYCLES (clock cycles summed over SIMDs) SQ_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU
#          SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 (quad-cycles with two VALU issued) SQ_WAVE_CYCLES
#          SQ_INSTS_SALU + GRBM_GUI_ACTIVE (effective clock = GRBM_GUI_ACTIVE / 8 / kernel wall)
#   lds  : SQ_CYCLES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT
#          SQ_INST_LEVEL_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL + GRBM_GUI_ACTIVE
# each with --kernel-trace (the kernel's own duration in the same run).
# usage: tools/pmc_r04.sh <outdir> [c4 hard1m min ...]   then: python3 tools/pmc_pipe_summary.py <outdir>
set -o pipefail
out=$1; shift; root=$(pwd); mkdir -p "$out"; export TMPDIR=/tmp
passes=${*:-c4 hard1m min}
OFF="--c2-puzzles 0 --minimal-puzzles 0 --hard-leg 0 --count-leg 0 --lane-puzzles 0 --cpu-seconds 0 --http-requests 0 --pmc-summary="
C4="$root/bench.py --steps 2 --warmup 1 --check-boards 0 $OFF"
HARD1M="$root/tools/solve_profile.py --workload hard --n 1000000 --reps 2 --donate 0 --solver quad"
MIN="$root/tools/solve_profile.py --workload minimal --n 1048576 --reps 2 --donate 0 --solver quad"
PIPE="SQ_CYCLES SQ_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVE_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
LDS="SQ_CYCLES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_INST_LEVEL_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL GRBM_GUI_ACTIVE"
run() {  # <tag> <counters> <program...>
  local tag=$1 ctr=$2; shift 2
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$root/$out/$tag" -o run -- "$@" \
     > "$root/$out/$tag.log" 2>&1) || { echo "pass $tag failed"; tail -5 "$out/$tag.log"; exit 1; }
  echo "pass $tag ok"
}
for p in $passes; do
  case $p in
  c4)     run c4_pipe "$PIPE" python3 $C4
          run c4_lds "$LDS" python3 $C4 ;;
  hard1m) run hard1m_pipe "$PIPE" python3 $HARD1M
          run hard1m_lds "$LDS" python3 $HARD1M ;;
  min)    run min_pipe "$PIPE" python3 $MIN
          run min_lds "$LDS" python3 $MIN ;;
  *) echo "unknown pass $p"; exit 2 ;;
  esac
done
python3 tools/pmc_pipe_summary.py "$out"
