#!/bin/bash
# Round profiles of the headline bench command per config (CONFIGS, default "c2 c3 c5"):
# rocprofv3 kernel trace + stats, then FETCH_SIZE and WRITE_SIZE PMC passes (one counter group per
# run, kernel trace only; the analyses on one stream - --serial - so the dispatch order is program
# order for scripts/pmc_traffic.py), each under its own time limit; stops at the first failure.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out
for c in ${CONFIGS:-c2 c3 c5}; do
  st=20; [ $c != c2 ] && st=3
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o run -- python3 -u bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline > $O/prof_$c.log 2>&1 || exit $?
  echo "trace $c ok"
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc_${c}_$ctr -o run -- python3 -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --probe-steps 1 --serial > $O/pmc_${c}_$ctr.log 2>&1 || exit $?
    echo "pmc $c $ctr ok"
  done
done
echo done
