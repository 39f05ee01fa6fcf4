#!/bin/bash
# SQ counter passes over the solve kernel (one rocprofv3 --pmc run per pass), run on the GPU box.
# usage: tools/solve_pmc.sh <outdir> [workload] [solver]
set -o pipefail
out=$1; wl=${2:-solve17}; sv=${3:-halfwave}
root=$(pwd)
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/solve_profile.py --stats --workload $wl --solver $sv > "$out/solve_stats.txt" 2>&1 || { cat "$out/solve_stats.txt"; exit 1; }
cat "$out/solve_stats.txt"
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS" \
            "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
            "SQ_LDS_IDX_ACTIVE SQ_BUSY_CU_CYCLES SQ_INST_CYCLES_VALU SQ_INSTS_VALU_INT32" \
            "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d "$root/$out/pass$i" -o run -- \
     python3 "$root/tools/solve_profile.py" --workload $wl --solver $sv --reps 1 > "$root/$out/pass$i.log" 2>&1) \
     || { echo "pass $i failed"; tail -5 "$out/pass$i.log"; exit 1; }
done
python3 tools/pmc_table.py "$out" | tee "$out/pmc_table.txt"
