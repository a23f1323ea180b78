#!/bin/bash
# round-3 GPU session B: parity of the series / RQ2 / RQ4 paths after kernel changes, c3 + c5
# benches, a serial c3 kernel trace for per-stage attribution
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=${TAG:-r3b}
[ -n "$NOTEST" ] || timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread -k "${PYK:-rq2 or rq4 or fullsize or rankstress or segsort or prims or graph or scale}" > $O/${T}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; [ -n "$NOTEST" ] || tail -3 $O/${T}_pytest.log
[ $rc -ne 0 ] && exit $rc
for c in ${CONFIGS:-c3 c5}; do
  timeout -k 10 600 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > $O/${T}_$c.json 2> $O/${T}_$c.err || exit $?
  python3 -c "import json; d=json.loads([l for l in open('$O/${T}_$c.json') if l.startswith('{')][-1]); print('$c', d['ms_per_step'])"
done
if [ -n "$TRACE" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/${T}_trace_$TRACE -o run -- python3 -u bench.py --config $TRACE --serial --steps 2 --warmup 1 --no-cpu-baseline --probe-steps 0 > $O/${T}_trace.log 2>&1 || exit $?
  echo trace ok
fi
