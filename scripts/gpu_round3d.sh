#!/bin/bash
# round-3 GPU session D: full GPU suite, c2 bench, c2 sharded (threaded drivers) bench, c3 / c5
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=${TAG:-r3d}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread ${PYK:+-k "$PYK"} > $O/${T}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/${T}_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/${T}_c2.json 2> $O/${T}_c2.err || exit $?
python3 -c "import json; d=json.loads([l for l in open('$O/${T}_c2.json') if l.startswith('{')][-1]); print('c2', d['ms_per_step'])"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --force-sharded > $O/${T}_c2fs.json 2> $O/${T}_c2fs.err || exit $?
python3 -c "import json; d=json.loads([l for l in open('$O/${T}_c2fs.json') if l.startswith('{')][-1]); print('c2 force-sharded', d['ms_per_step'])"
for c in ${CONFIGS:-c3 c5}; do
  timeout -k 10 600 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > $O/${T}_$c.json 2> $O/${T}_$c.err || exit $?
  python3 -c "import json; d=json.loads([l for l in open('$O/${T}_$c.json') if l.startswith('{')][-1]); print('$c', d['ms_per_step'])"
done
if [ -n "$TRACE" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/${T}_trace_$TRACE -o run -- python3 -u bench.py --config $TRACE --serial --steps 2 --warmup 1 --no-cpu-baseline --probe-steps 0 > $O/${T}_trace.log 2>&1 || exit $?
  echo trace ok
fi
