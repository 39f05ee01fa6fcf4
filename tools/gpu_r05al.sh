#!/bin/bash
# round 5 box pass 41: evidence of the final build -- PMC (traffic + pipe/LDS), GPU suite, smoke,
# rocprof kernel stats of the C3 and C4 commands, then the default bench with the fresh PMC records
set -o pipefail
bash tools/pmc_c4.sh gpurun_out/r05al/c4 > gpurun_out/r05al_pmc_c4.log 2>&1 || { tail -20 gpurun_out/r05al_pmc_c4.log; exit 1; }
bash tools/pmc_r04.sh gpurun_out/r05al/pipe c4 hard1m min > gpurun_out/r05al_pmc_pipe.log 2>&1 || { tail -20 gpurun_out/r05al_pmc_pipe.log; exit 1; }
cp gpurun_out/r05al/c4/pmc_c4.json profiles/r05/pmc_c4.json
cp gpurun_out/r05al/pipe/pmc_pipe.json profiles/r05/pmc_pipe.json
grep "^c4\|^hard1m\|^min" gpurun_out/r05al_pmc_pipe.log | cut -c1-300
bash tools/gpu_round.sh r05al tests prof_c3 prof_c4 bench > gpurun_out/r05al.log 2>&1 || { tail -30 gpurun_out/r05al.log; exit 1; }
tail -3 gpurun_out/r05al/pytest_gpu.log
