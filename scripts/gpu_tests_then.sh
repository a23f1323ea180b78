#!/bin/bash
# A subset of the GPU tests (TESTS=files), then the sharded step at world 1 (CONFIGS; serial and
# threaded drivers) and the single-table step for comparison
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=${TAG:-r3h}
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 500 --timeout-method thread > $O/${T}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/${T}_pytest.log
[ $rc -ne 0 ] && exit $rc
for c in ${CONFIGS:-c2 c3}; do
  st=20; [ $c != c2 ] && st=5
  for mode in "--force-sharded --serial" "--force-sharded" "--force-sharded --shard-graphs" ""; do
    timeout -k 10 300 python -u bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline --probe-steps 0 $mode > $O/${T}_b.json 2> $O/${T}_b.err || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$O/${T}_b.json') if l.startswith('{')][-1]); print('$c [$mode]', d['ms_per_step'], d['config'].get('driver_host_ms', ''), flush=True)"
  done
done
for c in $TRACES; do
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/${T}_trace_$c -o run -- python3 -u bench.py --config $c --force-sharded --serial --steps 2 --warmup 1 --no-cpu-baseline --probe-steps 0 > $O/${T}_trace_$c.log 2>&1 || exit $?
  echo "sharded trace $c ok"
done
