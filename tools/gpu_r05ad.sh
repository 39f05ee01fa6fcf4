#!/bin/bash
# round 5 box pass 34: PMC evidence of the current build -- traffic / SQ of C4 and C3 (pmc_c4.sh), per-SIMD
# pipe and LDS of prop32 on C4 and of solve4 on hard 1M and minimal 1M (pmc_r04.sh)
set -o pipefail
bash tools/pmc_c4.sh gpurun_out/r05ad/c4 || exit 1
bash tools/pmc_r04.sh gpurun_out/r05ad/pipe c4 hard1m min || exit 1
