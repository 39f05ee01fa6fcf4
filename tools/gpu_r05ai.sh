#!/bin/bash
# round 5 box pass 38: what bounds the split phase of the phased hard-1M solve (solve4_kernel<false,...>
# after the prop32 pass): per-SIMD pipe, LDS and SQ wait counters, one pass each
set -o pipefail
out=gpurun_out/r05ai
mkdir -p $out
export TMPDIR=/tmp
root=$(pwd)
CMD="$root/tools/solve_profile.py --solver quad --workload hard --n 1000000 --reps 2 --donate 1 --donate-max 0"
PIPE="SQ_CYCLES SQ_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVE_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
LDS="SQ_CYCLES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_INST_LEVEL_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL GRBM_GUI_ACTIVE"
WAIT="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM"
for pass in pipe lds wait; do
  case $pass in pipe) ctr="$PIPE";; lds) ctr="$LDS";; wait) ctr="$WAIT";; esac
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$root/$out/hard1m_$pass" -o run -- python3 $CMD > "$root/$out/$pass.log" 2>&1) || { echo "pass $pass failed"; tail -5 $out/$pass.log; exit 1; }
  echo "pass $pass ok"
done
PMC_SEARCH_KERNEL="solve4_kernel<false" python3 tools/pmc_pipe_summary.py $out | grep hard1m
python3 tools/pmc_sq_sum.py $out/hard1m_wait | grep "solve4_kernel<false" | head -4
