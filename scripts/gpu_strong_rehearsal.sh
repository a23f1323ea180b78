#!/bin/bash
# Strong-scaling rehearsal on one GPU: the config-3 table cut by parallel.shard_bounds into N shards;
# the sharded step of shard 0 and shard N-1 at world 1 (per-rank compute, no exchange)
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out; mkdir -p $O
C=${CONFIG:-c3}
# RANKS=all: every shard (a table whose largest project makes one shard the slowest)
for n in ${NS:-1 2 4 8}; do
  ranks="0 $((n - 1))"; [ "${RANKS:-}" = all ] && ranks=$(seq 0 $((n - 1)))
  for r in $ranks; do
    [ $n = 1 ] && [ $r != 0 ] && continue
    timeout -k 10 300 python -u bench.py --config $C --steps 10 --warmup 2 --no-cpu-baseline --probe-steps 0 --strong --force-sharded --shard-of $n --shard-rank $r > $O/sr.json 2> $O/sr.err || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$O/sr.json') if l.startswith('{')][-1]); print('$C shard $r of $n', d['ms_per_step'], d['config']['rows_per_rank'], flush=True)"
  done
done
