#!/bin/bash
# VALU/LDS issue-rate calibration + the SQ counters of the same kernels (run on the GPU box).
# usage: tools/calib_pmc.sh <outdir>
set -o pipefail
out=$1; root=$(pwd); mkdir -p "$out"; export TMPDIR=/tmp
timeout -k 10 60 ./tools/valu_calib > "$out/calib.txt" 2>&1 || { cat "$out/calib.txt"; exit 1; }
cat "$out/calib.txt"
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CU_CYCLES SQ_INST_CYCLES_VALU" \
            "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 60 rocprofv3 --pmc $pass --output-format csv -d "$root/$out/pass$i" -o run -- \
     "$root/tools/valu_calib" > "$root/$out/pass$i.log" 2>&1) || { echo "pass $i failed"; tail -5 "$out/pass$i.log"; exit 1; }
done
python3 tools/pmc_table.py "$out" --all | tee "$out/pmc_table.txt"
