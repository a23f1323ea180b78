#!/bin/bash
# Quick GPU iteration: selected parity tests, then the bench at the given configs (store-only and
# full step).  TESTS (pytest -k/-file args), CONFIGS (e.g. "c2 c3 c5"), FULL (configs run with all stages).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TESTS=${TESTS:-tests/test_gpu_scale.py tests/test_gpu_rq1.py tests/test_gpu_rq2.py tests/test_gpu_rq3.py tests/test_gpu_rq4.py}
if [ "$TESTS" != none ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/pytest_quick.log 2>&1
  rc=$?; echo "pytest rc $rc"; tail -3 $OUT/pytest_quick.log; grep -E "FAILED|Error" $OUT/pytest_quick.log | head -10
  [ $rc -ne 0 ] && exit $rc
fi
for c in ${CONFIGS:-c2}; do
  st=3; [ $c = c2 ] && st=20
  timeout -k 10 400 python -u bench.py --config $c --stages store --steps $st --warmup 1 --no-cpu-baseline --probe-steps 3 > $OUT/bstore_$c.log 2>&1 || exit $?
  echo "store $c $(grep -o '"ms_per_step": [0-9.]*' $OUT/bstore_$c.log | head -1)"
done
for c in ${FULL:-c2}; do
  st=3; [ $c = c2 ] && st=20
  timeout -k 10 400 python -u bench.py --config $c --steps $st --warmup 1 --no-cpu-baseline > $OUT/bfull_$c.log 2>&1 || exit $?
  echo "full $c $(grep -o '"ms_per_step": [0-9.]*' $OUT/bfull_$c.log | head -1)"
done
echo done
