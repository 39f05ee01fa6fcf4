#!/bin/bash
# round 5 box pass 1: the instruction-mix ceilings of solve4's compute roofline
# (tools/issue_calib at 7 and 8 waves per SIMD, timed and under PMC), the per-part cycle breakdown of
# the C4 launch (profiling build), and fresh per-SIMD pipe / LDS and HBM traffic counters of this
# round's build.
set -o pipefail
out=gpurun_out/r05a
mkdir -p $out
export TMPDIR=/tmp
root=$(pwd)
timeout -k 10 120 tools/issue_calib > $out/issue_calib.txt 2>&1 || { tail -20 $out/issue_calib.txt; exit 1; }
cat $out/issue_calib.txt
PIPE="SQ_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
WAIT="SQ_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
for p in pipe wait; do
  ctr=$PIPE; [ $p = wait ] && ctr=$WAIT
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $root/$out/calib/$p -o run -- \
     $root/tools/issue_calib > $root/$out/calib_$p.log 2>&1) || { echo "calib pmc $p failed"; tail -5 $out/calib_$p.log; exit 1; }
  echo "calib pmc $p ok"
done
python3 tools/issue_calib_summary.py $out/calib pipe wait
SDK_LIB_PATH=$root/build/variants/lib_prof.so timeout -k 10 180 python tools/solve4_prof.py --n 10000000 > $out/prof_parts_c4.txt 2>&1 \
  || { tail -20 $out/prof_parts_c4.txt; exit 1; }
cat $out/prof_parts_c4.txt
SDK_LIB_PATH=$root/build/variants/lib_prof.so timeout -k 10 180 python tools/solve4_prof.py --n 1048576 --workload minimal > $out/prof_parts_min.txt 2>&1 \
  || { tail -20 $out/prof_parts_min.txt; exit 1; }
cat $out/prof_parts_min.txt
timeout -k 10 600 bash tools/pmc_r04.sh $out/pmc c4 > $out/pmc.log 2>&1 || { tail -30 $out/pmc.log; exit 1; }
tail -4 $out/pmc.log
timeout -k 10 600 bash tools/pmc_c4.sh $out/traffic > $out/traffic.log 2>&1 || { tail -30 $out/traffic.log; exit 1; }
tail -12 $out/traffic.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_solve.py \
  -k "frontier_first or two_rank or rccl or clique" > $out/pytest_first.log 2>&1 || { tail -40 $out/pytest_first.log; exit 1; }
tail -12 $out/pytest_first.log
