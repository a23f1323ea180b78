#!/bin/bash
# A/B of the sharded step's host threading on one box (world 1, RCCL): serial drivers, one thread
# per stream group, one thread per driver
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out; mkdir -p $O
run() {
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --force-sharded --probe-steps 0 "$@" > $O/sab.json 2> $O/sab.err || exit $?
  python3 -c "import json; d=json.loads([l for l in open('$O/sab.json') if l.startswith('{')][-1]); print('$*', d['ms_per_step'], flush=True)"
}
for r in 1 2; do
  run --serial
  run
  run --shard-groups "rq3|rq4b|rq2_count|rq1|rq4a|rq2_add"
  run --shard-groups "rq3,rq4b|rq2_count,rq1,rq4a,rq2_add"
done
