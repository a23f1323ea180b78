#!/bin/bash
# The sharded step at world 1 (RCCL): per-stage step times, then a serial kernel trace of c2 and c3
# (scripts/stage_breakdown.py cuts it per driver: kernel busy time vs span = host gaps)
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=${TAG:-shtr}
for c in ${CONFIGS:-c2 c3}; do
  st=20; [ $c != c2 ] && st=5
  timeout -k 10 300 python -u bench.py --config $c --force-sharded --serial --steps $st --warmup 2 --no-cpu-baseline --probe-steps 0 > $O/${T}_$c.json 2> $O/${T}_$c.err || exit $?
  python3 -c "import json; d=json.loads([l for l in open('$O/${T}_$c.json') if l.startswith('{')][-1]); print('$c sharded serial', d['ms_per_step'], flush=True)"
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/${T}_trace_$c -o run -- python3 -u bench.py --config $c --force-sharded --serial --steps 2 --warmup 1 --no-cpu-baseline --probe-steps 0 > $O/${T}_trace_$c.log 2>&1 || exit $?
  echo "trace $c ok"
done
