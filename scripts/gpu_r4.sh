#!/bin/bash
# Round-4 GPU session helper: STEPS selects among
#   prof:<cfg>   rocprofv3 kernel trace + stats of the headline bench command on <cfg>
#   stages:<cfg> per-stage step times (serial), stage_times.sh
#   drop:<cfg>   the concurrent step without one analysis group at a time
#   bench:<cfg>  one bench line (json) on <cfg>
#   tests[:k]    pytest -m gpu (optionally -k expression)
# Each GPU step has its own time limit; a fault / abort / timeout ends the script.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=${TAG:-r4}
for s in $STEPS; do
  kind=${s%%:*}; arg=${s#*:}
  case $kind in
    prof)
      st=20; [ "$arg" != c2 ] && st=3
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_$arg -o run -- python3 -u bench.py --config $arg --steps $st --warmup 2 --no-cpu-baseline > $O/${T}_prof_$arg.log 2>&1 || exit $?
      f=$(ls $O/${T}_prof_$arg/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find $O/${T}_prof_$arg -name "*kernel_stats.csv" | head -1)
      python3 scripts/kstats.py "$f" $((st + 3)) 40 > $O/${T}_kstats_$arg.txt; head -30 $O/${T}_kstats_$arg.txt ;;
    stages)
      CONFIG=$arg timeout -k 10 900 bash scripts/stage_times.sh > $O/${T}_stages_$arg.txt 2>&1 || exit $?; cat $O/${T}_stages_$arg.txt ;;
    drop)
      CONFIG=$arg DROP=1 timeout -k 10 900 bash scripts/stage_times.sh > $O/${T}_drop_$arg.txt 2>&1 || exit $?; cat $O/${T}_drop_$arg.txt ;;
    bench)
      st=20; [ "$arg" != c2 ] && st=5
      timeout -k 10 600 python -u bench.py --config $arg --steps $st --warmup 2 --no-cpu-baseline > $O/${T}_bench_$arg.json 2> $O/${T}_bench_$arg.err || exit $?
      python3 -c "import json; d=json.loads([l for l in open('$O/${T}_bench_$arg.json') if l.startswith('{')][-1]); print('$arg', d['ms_per_step'], flush=True)" ;;
    tests)
      k=""; [ "$arg" != tests ] && k="${arg//+/ or }"
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread ${k:+-k "$k"} > $O/${T}_pytest.log 2>&1; rc=$?
      echo "pytest rc=$rc"; tail -3 $O/${T}_pytest.log; [ $rc -ne 0 ] && exit $rc ;;
  esac
done
echo done
