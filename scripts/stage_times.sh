#!/bin/bash
# Per-stage step time on the GPU: the store build alone, then store + one analysis at a time
# (EXTRA="--force-sharded" for the project-sharded step path).
cd "$(dirname "$0")/.." || exit 1
for st in store store,rq1 store,rq2_count store,rq2_add store,rq3 store,rq4a store,rq4b; do
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline $EXTRA --stages $st > gpurun_out/stage.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/stage.json') if l.startswith('{')][-1]); print('$st', d['ms_per_step'])"
done
