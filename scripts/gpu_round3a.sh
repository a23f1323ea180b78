#!/bin/bash
# round-3 GPU session A: parity of the RQ4b / full-size paths, c3/c5 CPU baselines, c3 stage times,
# c2 kernel trace (timeline of one step)
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread -k "rq4 or fullsize or sharded_c3 or rankstress or graph" > $O/r3a_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/r3a_pytest.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 900 python -u bench.py --config c3 --steps 5 --warmup 2 > $O/r3a_c3.json 2> $O/r3a_c3.err || exit $?
echo c3 ok; tail -c 600 $O/r3a_c3.json
timeout -k 10 900 python -u bench.py --config c5 --steps 5 --warmup 2 > $O/r3a_c5.json 2> $O/r3a_c5.err || exit $?
echo c5 ok
CONFIG=c3 NSTEPS=5 timeout -k 10 900 bash scripts/stage_times.sh > $O/r3a_stages_c3.txt 2>&1 || exit $?
cat $O/r3a_stages_c3.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/r3a_trace_c2 -o run -- python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --probe-steps 0 > $O/r3a_trace_c2.log 2>&1 || exit $?
echo trace ok
