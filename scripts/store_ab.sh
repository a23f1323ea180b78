#!/bin/bash
# Store-build step alone (--stages store, the concurrent step's store with its helper streams) and
# the whole step, with and without the helper fork (FZ_STORE_FORK=0), same box, alternating.
# usage: CONFIG=c2 scripts/store_ab.sh
cd "$(dirname "$0")/.." || exit 1
C=${CONFIG:-c2}
for r in 1 2; do
  for f in 1 0; do
    for st in store store,rq1,rq2_count,rq2_add,rq3,rq4a,rq4b; do
      FZ_STORE_FORK=$f timeout -k 10 300 python -u bench.py --config $C --steps 40 --warmup 3 --no-cpu-baseline --probe-steps 0 --stages $st > gpurun_out/store_ab.json 2>/dev/null || exit $?
      python3 -c "import json; d=json.loads([l for l in open('gpurun_out/store_ab.json') if l.startswith('{')][-1]); print('$C fork=$f $st', d['ms_per_step'], flush=True)"
    done
  done
done
