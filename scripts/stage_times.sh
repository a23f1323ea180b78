#!/bin/bash
# Per-stage step time on the GPU: the store build alone, then store + one analysis at a time
# (CONFIG=c3 for another table, EXTRA="--force-sharded" for the project-sharded step path).
cd "$(dirname "$0")/.." || exit 1
C=${CONFIG:-c2}
N=${NSTEPS:-20}
for st in store store,rq1 store,rq2_count store,rq2_add store,rq3 store,rq4a store,rq4b; do
  timeout -k 10 300 python -u bench.py --config $C --steps $N --warmup 2 --no-cpu-baseline --probe-steps 0 --serial $EXTRA --stages $st > gpurun_out/stage.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/stage.json') if l.startswith('{')][-1]); print('$C $st', d['ms_per_step'], flush=True)"
done
