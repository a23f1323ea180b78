#!/bin/bash
# A/B of the sharded step's local phases: per driver (default) vs all at once on four streams
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out; mkdir -p $O
run() {
  local c=$1 st=$2; shift 2
  timeout -k 10 300 python -u bench.py --config $c --steps $st --warmup 3 --no-cpu-baseline --probe-steps 0 --force-sharded "$@" > $O/sla.json 2> $O/sla.err || exit $?
  python3 -c "import json; d=json.loads([l for l in open('$O/sla.json') if l.startswith('{')][-1]); print('$c $*', d['ms_per_step'], flush=True)"
}
for r in 1 2; do
  run c2 100
  run c2 100 --shard-local streams
done
for r in 1 2; do
  run c3 10
  run c3 10 --shard-local streams
done
run c3 10 --strong --shard-of 8 --shard-local streams
run c3 10 --strong --shard-of 8
