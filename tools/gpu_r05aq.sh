#!/bin/bash
# round 5 box pass 45: per-SIMD pipe / LDS PMC of the final prop32 build (C4), for the bench's roofline.valu
set -o pipefail
bash tools/pmc_r04.sh gpurun_out/r05aq/pipe c4 hard1m min > gpurun_out/r05aq_pmc_pipe.log 2>&1 || { tail -20 gpurun_out/r05aq_pmc_pipe.log; exit 1; }
grep "^c4\|^hard1m\|^min" gpurun_out/r05aq_pmc_pipe.log | cut -c1-260
