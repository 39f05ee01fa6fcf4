#!/bin/bash
# round 4 box pass: the driver's multi-rank launch path rehearsed on one GPU -- torchrun, two
# ranks sharing the card, the default bench legs (a shared GPU halves each rank's share: the
# numbers are not scaling evidence, the run is)
set -o pipefail
out=gpurun_out/r04aa
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > $out/bench_2rank.json 2> $out/bench_2rank.err \
  || { tail -30 $out/bench_2rank.err; exit 1; }
tail -c 1500 $out/bench_2rank.json
