#!/bin/bash
# rocprofv3 kernel trace of store-only bench steps (CONFIGS), one directory per config.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
for c in ${CONFIGS:-c2}; do
  st=5; [ $c != c2 ] && st=2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_store_$c -o run -- python -u bench.py --config $c --stages ${STAGES:-store} --steps $st --warmup 1 --no-cpu-baseline --probe-steps 0 > gpurun_out/prof_store_$c.log 2>&1 || exit $?
done
