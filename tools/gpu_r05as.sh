#!/bin/bash
# round 5 box pass 46: the N = 2 rank path on one GPU (two ranks share the card; RCCL legs skipped)
# with prop32 and three passes in flight (the default) -- the driver's torchrun command shape
set -o pipefail
out=gpurun_out/r05as
mkdir -p $out
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > $out/bench_2rank.json 2> $out/bench_2rank.err \
  || { tail -30 $out/bench_2rank.err; exit 1; }
python3 -c "
import json; r=json.loads(open('$out/bench_2rank.json').read().strip().splitlines()[-1])
print('n_gpus', r['n_gpus'], 'value', r['value'], 'parity', r['parity'], 'single', r['single_stream']['value'])
print('weak', {k: r.get('weak_scaling',{}).get(k) for k in ('value','parity')})
print('hard', {k: round(r['hard_search'][k]['donation']['value']/1e6,1) for k in ('hard_100k','hard_1m')} if 'hard_search' in r and 'hard_100k' in r['hard_search'] else r.get('hard_search'))
print('c5', r.get('c5_count'))
print('keys', list(r.keys())[-4:])
"
