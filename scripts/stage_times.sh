#!/bin/bash
# Per-stage step time on the GPU: the store build alone, then store + one analysis at a time
# (CONFIG=c3 for another table, EXTRA="--force-sharded" for the project-sharded step path).
# DROP=1: the concurrent graph step with all analyses, then without one group at a time (the
# marginal cost of each group on the critical path).
cd "$(dirname "$0")/.." || exit 1
C=${CONFIG:-c2}
N=${NSTEPS:-20}
if [ -n "$DROP" ]; then
  SETS="store,rq1,rq2_count,rq2_add,rq3,rq4a,rq4b store,rq1,rq2_count,rq2_add,rq4a,rq4b store,rq1,rq2_count,rq2_add,rq3,rq4a store,rq1,rq2_add,rq3,rq4a,rq4b store,rq2_count,rq3,rq4b store"
  SER=""
else
  SETS="store store,rq1 store,rq2_count store,rq2_add store,rq3 store,rq4a store,rq4b"
  SER="--serial"
fi
for st in $SETS; do
  timeout -k 10 300 python -u bench.py --config $C --steps $N --warmup 2 --no-cpu-baseline --probe-steps 0 $SER $EXTRA --stages $st > gpurun_out/stage.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/stage.json') if l.startswith('{')][-1]); print('$C $st', d['ms_per_step'], flush=True)"
done
