#!/bin/bash
# A/B of pipelined steps (bench.py --lanes) against HIP hardware queues per process, two rounds
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out; mkdir -p $O
run() {
  local c=$1 q=$2 l=$3 st=$4
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --config $c --steps $st --warmup 3 --no-cpu-baseline --probe-steps 0 --lanes $l > $O/lab.json 2> $O/lab.err || exit $?
  python3 -c "import json; d=json.loads([l for l in open('$O/lab.json') if l.startswith('{')][-1]); print('$c queues=$q lanes=$l', d['ms_per_step'], flush=True)"
}
for r in 1 2; do
  run c2 4 1 100
  run c2 4 2 100
  run c2 8 2 100
  run c2 8 1 100
done
for r in 1 2; do
  run c3 4 1 10
  run c3 4 2 10
  run c3 8 2 10
done
