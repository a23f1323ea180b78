#!/bin/bash
# A/B of the concurrent single-table step against the number of HIP hardware queues per process
# (GPU_MAX_HW_QUEUES, HIP's default 4) and the analysis groups (one stream each), two rounds
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out; mkdir -p $O
C=${CONFIG:-c2}
run() {
  local q=$1; shift
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --config $C --steps ${NSTEPS:-100} --warmup 3 --no-cpu-baseline --probe-steps 0 "$@" > $O/qab.json 2> $O/qab.err || exit $?
  python3 -c "import json; d=json.loads([l for l in open('$O/qab.json') if l.startswith('{')][-1]); print('$C queues=$q $*', d['ms_per_step'], flush=True)"
}
for r in 1 2; do
  run 4
  run 8
  run 8 --groups "rq3|rq4b|rq2_count|rq1|rq4a|rq2_add"
  run 8 --groups "rq3|rq4b|rq2_count|rq1,rq2_add|rq4a"
  run 4 --groups "rq3|rq4b|rq2_count|rq1|rq4a|rq2_add"
done
