#!/bin/bash
# scratch GPU step: concurrent-analysis parity, then serial vs concurrent bench at c2/c3
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_concurrent.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_conc.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -3 $OUT/pytest_conc.log; [ $rc -ne 0 ] && exit $rc
for c in c2 c3; do
  st=3; [ $c = c2 ] && st=30
  timeout -k 10 300 python -u bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline --serial > $OUT/bser_$c.log 2>&1 || exit $?
  echo "serial $c $(grep -o '"ms_per_step": [0-9.]*' $OUT/bser_$c.log | head -1)"
  timeout -k 10 300 python -u bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline > $OUT/bconc_$c.log 2>&1 || exit $?
  echo "conc $c $(grep -o '"ms_per_step": [0-9.]*' $OUT/bconc_$c.log | head -1)"
done
echo done
