#!/bin/bash
# One rocprofv3 PMC pass per counter group over a short bench (run on the GPU box).
# usage: tools/pmc_pass.sh <outdir> <tag> <counters...>
set -o pipefail
out=$1; tag=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d "$out" -o "$tag" -- \
  python3 bench.py --steps 2 --warmup 0 --check-steps 2 --cpu-seconds 0 --batch 2000000 --check-boards 50000000
