#!/bin/bash
# Round-end measurement of the current tree (one gpurun call per CONFIGS group): per config
#   pmc  - FETCH_SIZE / WRITE_SIZE passes of bench.py --serial (separate runs, kernel trace only),
#          scripts/pmc_traffic.py -> profiles/${TAG}_<c>_pmc_traffic.json (read by the bench line)
#   bench- the bench line with the CPU baseline -> gpurun_out/${TAG}_<c>_bench.json
#   prof - rocprofv3 --kernel-trace --stats of the bench command -> kernel stats + kstats summary
# STEPS selects (default "pmc bench prof"); each GPU step under its own time limit; the first
# failure ends the script.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=${TAG:-r06f}
for c in ${CONFIGS:-c2}; do
  st=20; [ $c != c2 ] && st=10
  for s in ${STEPS:-pmc bench prof}; do
    case $s in
      pmc)
        for ctr in FETCH_SIZE WRITE_SIZE; do
          timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d $O/${T}_pmc_${c}_$ctr -o run -- python3 -u bench.py \
            --config $c --steps 2 --warmup 1 --no-cpu-baseline --probe-steps 1 --serial > $O/${T}_pmc_${c}_$ctr.log 2>&1 \
            || { echo "pmc $c $ctr failed"; tail -3 $O/${T}_pmc_${c}_$ctr.log; exit 1; }
        done
        python3 scripts/pmc_traffic.py $(find $O/${T}_pmc_${c}_FETCH_SIZE -name "*counter_collection.csv" | head -1) \
          $(find $O/${T}_pmc_${c}_WRITE_SIZE -name "*counter_collection.csv" | head -1) $c \
          profiles/${T}_${c}_pmc_traffic.json > /dev/null && cp profiles/${T}_${c}_pmc_traffic.json $O/ && echo "pmc $c ok" ;;
      bench)
        timeout -k 10 ${BENCH_S:-420} python3 -u bench.py --config $c --steps $st --warmup 3 > $O/${T}_${c}_bench.json \
          2> $O/${T}_${c}_bench.err || { echo "bench $c failed"; tail -5 $O/${T}_${c}_bench.err; exit 1; }
        echo "bench $c $(grep -o '"ms_per_step": [0-9.]*' $O/${T}_${c}_bench.json | head -1)" ;;
      prof)
        timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_$c -o run -- python3 -u bench.py \
          --config $c --steps $st --warmup 2 --no-cpu-baseline > $O/${T}_prof_$c.log 2>&1 || { echo "prof $c failed"; exit 1; }
        python3 scripts/kstats.py $(find $O/${T}_prof_$c -name '*kernel_stats.csv' | head -1) auto 40 > $O/${T}_kstats_$c.txt
        cp $(find $O/${T}_prof_$c -name '*kernel_stats.csv' | head -1) $O/${T}_${c}_kernel_stats.csv
        head -3 $O/${T}_kstats_$c.txt ;;
    esac
  done
done
echo done
