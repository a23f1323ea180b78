#!/bin/bash
# full GPU parity suite, then the c2 bench twice (variance) and optionally CONFIGS benches
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -1 $O/pytest_gpu.log; grep -E "FAILED" $O/pytest_gpu.log | head -5; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 50 --warmup 3 --no-cpu-baseline --probe-steps 0 > $O/btb_$i.log 2>&1 || exit $?
  echo "c2 $i $(grep -o '"ms_per_step": [0-9.]*' $O/btb_$i.log)"
done
for c in $CONFIGS; do
  timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --probe-steps 0 > $O/btb_$c.log 2>&1 || exit $?
  echo "$c $(grep -o '"ms_per_step": [0-9.]*' $O/btb_$c.log)"
done
echo done
