#!/bin/bash
# same-box comparison of stream groupings (bench.py --groups), GROUPINGS separated by ';'
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out; mkdir -p $O
IFS=';' read -ra GL <<< "$GROUPINGS"
for r in 1 2; do
  k=0
  for g in "${GL[@]}"; do
    k=$((k+1))
    timeout -k 10 200 python -u bench.py --steps 50 --warmup 3 --no-cpu-baseline --probe-steps 0 --groups "$g" > $O/bg_${k}_$r.log 2>&1 || exit $?
    echo "$g $r $(grep -o '"ms_per_step": [0-9.]*' $O/bg_${k}_$r.log)"
  done
done
