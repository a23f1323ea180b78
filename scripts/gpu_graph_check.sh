#!/bin/bash
# Graph-replay check: the graph / concurrency parity tests, then the bench with and without graphs.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_concurrent.py tests/test_gpu_segsort.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_graph.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -3 $O/pytest_graph.log; [ $rc -ne 0 ] && exit $rc
for mode in "" "--no-graphs"; do
  timeout -k 10 300 python -u bench.py --steps 50 --warmup 3 --no-cpu-baseline --probe-steps 0 $mode > $O/bgraph$mode.log 2>&1 || exit $?
  echo "c2 $mode $(grep -o '"ms_per_step": [0-9.]*' $O/bgraph$mode.log)"
done
for c in ${CONFIGS:-c3}; do
  timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --probe-steps 0 > $O/bgraph_$c.log 2>&1 || exit $?
  echo "$c $(grep -o '"ms_per_step": [0-9.]*' $O/bgraph_$c.log)"
done
echo done
