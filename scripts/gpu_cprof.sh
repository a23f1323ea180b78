#!/bin/bash
# cProfile of the strong rehearsal's sharded step on given shards: SHARDS="2 5", CONFIG, N.
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out; mkdir -p $O
T=${TAG:-r6c}
for r in ${SHARDS:-2 5}; do
  timeout -k 10 300 python -u bench.py --config ${CONFIG:-c5L} --steps 10 --warmup 2 --no-cpu-baseline --probe-steps 0 \
    --strong --force-sharded --shard-of ${N:-8} --shard-rank $r --cprofile $O/${T}_cprof_$r.txt > $O/${T}_sr_$r.json 2> $O/${T}_sr_$r.err \
    || { tail -5 $O/${T}_sr_$r.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/${T}_sr_$r.json') if l.startswith('{')][-1]); print('shard $r', d['ms_per_step'], d['config'].get('driver_host_ms'))"
done
echo done
