#!/bin/bash
# A/B of the sharded step's host threading on one box (world 1, RCCL): the driver groups per host
# thread (bench.py --shard-groups), two rounds
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out; mkdir -p $O
C=${CONFIG:-c2}
run() {
  timeout -k 10 300 python -u bench.py --config $C --steps ${NSTEPS:-100} --warmup 3 --no-cpu-baseline --force-sharded --probe-steps 0 "$@" > $O/sab.json 2> $O/sab.err || exit $?
  python3 -c "import json; d=json.loads([l for l in open('$O/sab.json') if l.startswith('{')][-1]); print('$C $*', d['ms_per_step'], flush=True)"
}
for r in 1 2; do
  run --shard-groups "rq3,rq4b|rq2_count,rq1,rq4a,rq2_add"
  run --shard-groups "rq3|rq4b|rq2_count,rq1,rq4a,rq2_add"
  run --shard-groups "rq3|rq4b|rq2_count|rq1,rq4a,rq2_add"
  run --shard-groups "rq3,rq1|rq4b,rq4a|rq2_count,rq2_add"
  run --shard-groups "rq4b,rq1,rq2_add|rq3,rq2_count,rq4a"
done
