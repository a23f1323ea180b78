#!/bin/bash
# round-3 GPU session F: parity (full suite), c2/c3/c5 benches, c3 + c5 serial kernel traces
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=${TAG:-r3f}
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread ${PYK:+-k "$PYK"} > $O/${T}_pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 $O/${T}_pytest.log
  [ $rc -ne 0 ] && exit $rc
fi
for c in ${CONFIGS:-c2 c3 c5}; do
  st=20; [ $c != c2 ] && st=5
  timeout -k 10 600 python -u bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline > $O/${T}_$c.json 2> $O/${T}_$c.err || exit $?
  python3 -c "import json; d=json.loads([l for l in open('$O/${T}_$c.json') if l.startswith('{')][-1]); print('$c', d['ms_per_step'], flush=True)"
done
for c in ${TRACES:-c3 c5}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/${T}_trace_$c -o run -- python3 -u bench.py --config $c --serial --steps 2 --warmup 1 --no-cpu-baseline --probe-steps 0 > $O/${T}_trace_$c.log 2>&1 || exit $?
  echo "trace $c ok"
done
