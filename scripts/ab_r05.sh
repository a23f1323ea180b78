#!/bin/bash
# Same-box A/B of the sharded step (one shard of a strong rehearsal) between this tree and the
# round-5 final tree checked out in ./ab_r05 (git worktree; not committed): ROUNDS rounds.
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out; mkdir -p $O
T=${TAG:-r6ab}
A="--config ${CONFIG:-c3} --steps 10 --warmup 2 --no-cpu-baseline --probe-steps 0 --strong --force-sharded --shard-of ${N:-8} --shard-rank ${R:-0} $EXTRA"
for r in $(seq 1 ${ROUNDS:-2}); do
  (cd ab_r05 && timeout -k 10 300 python -u bench.py $A > ../$O/${T}_old.json 2> ../$O/${T}_old.err) || { tail -5 $O/${T}_old.err; exit 1; }
  timeout -k 10 300 python -u bench.py $A > $O/${T}_new.json 2> $O/${T}_new.err || { tail -5 $O/${T}_new.err; exit 1; }
  for v in old new; do
    python3 -c "import json; d=json.loads([l for l in open('$O/${T}_$v.json') if l.startswith('{')][-1]); print('$v r$r', d['ms_per_step'], d['config'].get('driver_host_ms'))" | tee -a $O/${T}.txt
  done
done
