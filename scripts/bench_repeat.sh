#!/bin/bash
# c2 bench repeated on one box (variance check): graphs x3, no graphs x2
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 50 --warmup 3 --no-cpu-baseline --probe-steps 0 ${EXTRA} > $O/brep_$i.log 2>&1 || exit $?
  echo "graphs $i $(grep -o '"ms_per_step": [0-9.]*' $O/brep_$i.log)"
done
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 50 --warmup 3 --no-cpu-baseline --probe-steps 0 --no-graphs ${EXTRA} > $O/brepn_$i.log 2>&1 || exit $?
  echo "nographs $i $(grep -o '"ms_per_step": [0-9.]*' $O/brepn_$i.log)"
done
