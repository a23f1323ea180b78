#!/bin/bash
# Round-4 GPU session helper: STEPS selects among
#   prof:<cfg>   rocprofv3 kernel trace + stats of the headline bench command on <cfg>
#   stages:<cfg> per-stage step times (serial), stage_times.sh
#   drop:<cfg>   the concurrent step without one analysis group at a time
#   bench:<cfg>  one bench line (json) on <cfg>
#   tests[:k]    pytest -m gpu (optionally -k expression, '+' = or)
#   pmc:<cfg> sq:<cfg> strong:<cfg> e2e:<cfg> cpu:<cfg>   PMC traffic, SQ counters, strong-scaling
#                rehearsal, end-to-end drop-ins, bench with the CPU baseline
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
      python3 scripts/kstats.py "$f" auto 40 > $O/${T}_kstats_$arg.txt; head -30 $O/${T}_kstats_$arg.txt ;;
    stages)
      CONFIG=$arg timeout -k 10 900 bash scripts/stage_times.sh > $O/${T}_stages_$arg.txt 2>&1 || exit $?; cat $O/${T}_stages_$arg.txt ;;
    st8)  # per-stage serial step times of shard 0 of 8 (the strong rehearsal's per-rank table)
      CONFIG=$arg EXTRA="--strong --shard-of 8 --shard-rank 0" timeout -k 10 900 bash scripts/stage_times.sh > $O/${T}_st8_$arg.txt 2>&1 || exit $?; cat $O/${T}_st8_$arg.txt ;;
    drop8)  # the concurrent step of shard 0 of 8 without one analysis group at a time
      CONFIG=$arg DROP=1 EXTRA="--strong --shard-of 8 --shard-rank 0" timeout -k 10 900 bash scripts/stage_times.sh > $O/${T}_drop8_$arg.txt 2>&1 || exit $?; cat $O/${T}_drop8_$arg.txt ;;
    drop)
      CONFIG=$arg DROP=1 timeout -k 10 900 bash scripts/stage_times.sh > $O/${T}_drop_$arg.txt 2>&1 || exit $?; cat $O/${T}_drop_$arg.txt ;;
    bench)
      st=20; [ "$arg" != c2 ] && st=5
      timeout -k 10 600 python -u bench.py --config $arg --steps $st --warmup 2 --no-cpu-baseline > $O/${T}_bench_$arg.json 2> $O/${T}_bench_$arg.err || exit $?
      python3 -c "import json; d=json.loads([l for l in open('$O/${T}_bench_$arg.json') if l.startswith('{')][-1]); print('$arg', d['ms_per_step'], flush=True)" ;;
    pmc)  # FETCH_SIZE and WRITE_SIZE in separate passes (serial analyses: program order), then traffic per probe
      for ctr in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d $O/${T}_pmc_${arg}_$ctr -o run -- python3 -u bench.py --config $arg --steps 2 --warmup 1 --no-cpu-baseline --probe-steps 1 --serial > $O/${T}_pmc_${arg}_$ctr.log 2>&1 || exit $?
      done
      python3 scripts/pmc_traffic.py $(find $O/${T}_pmc_${arg}_FETCH_SIZE -name "*counter_collection.csv" | head -1) $(find $O/${T}_pmc_${arg}_WRITE_SIZE -name "*counter_collection.csv" | head -1) $arg $O/${T}_${arg}_pmc_traffic.json > /dev/null && echo "pmc $arg ok" ;;
    calib)  # FETCH_SIZE / WRITE_SIZE per access width on known byte counts (scripts/pmc_calib.hip)
      for ctr in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $O/${T}_calib_$ctr -o run -- scripts/build/pmc_calib > $O/${T}_calib_$ctr.log 2>&1 || exit $?
      done
      python3 scripts/pmc_calib.py $(find $O/${T}_calib_FETCH_SIZE -name "*counter_collection.csv" | head -1) $(find $O/${T}_calib_WRITE_SIZE -name "*counter_collection.csv" | head -1) $O/${T}_calib_FETCH_SIZE.log $O/${T}_pmc_calib.json ;;
    pmck)  # counter bytes per kernel name of a serial step over some stages: pmck:<cfg>@<stages>[@<N>]
      IFS=@ read -r cfg sts nsh <<< "$arg"
      extra=""; [ -n "$nsh" ] && extra="--strong --shard-of $nsh --shard-rank 0"
      for ctr in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d $O/${T}_pmck_${cfg}_$ctr -o run -- python3 -u bench.py --config $cfg --steps 1 --warmup 1 --no-cpu-baseline --probe-steps 0 --serial --stages $sts $extra > $O/${T}_pmck_${cfg}_$ctr.log 2>&1 || exit $?
      done
      python3 scripts/pmc_by_kernel.py $(find $O/${T}_pmck_${cfg}_FETCH_SIZE -name "*counter_collection.csv" | head -1) $(find $O/${T}_pmck_${cfg}_WRITE_SIZE -name "*counter_collection.csv" | head -1) $O/${T}_pmck_$cfg.json > $O/${T}_pmck_$cfg.txt && head -25 $O/${T}_pmck_$cfg.txt ;;
    sq)  # shader-sequencer counters per kernel family (one pass, <= 8 SQ counters)
      timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VALU --output-format csv -d $O/${T}_sq_$arg -o run -- python3 -u bench.py --config $arg --steps 2 --warmup 1 --no-cpu-baseline --probe-steps 0 --serial > $O/${T}_sq_$arg.log 2>&1 || exit $?
      python3 scripts/pmc_sq.py $(find $O/${T}_sq_$arg -name "*counter_collection.csv" | head -1) $O/${T}_${arg}_sq.json ;;
    strong)
      CONFIG=${arg%%@*} RANKS=$([ "${arg#*@}" != "$arg" ] && echo all) timeout -k 10 1100 bash scripts/gpu_strong_rehearsal.sh > $O/${T}_strong_$arg.txt 2>&1 || exit $?; cat $O/${T}_strong_$arg.txt ;;
    e2e)
      timeout -k 10 900 python -u scripts/e2e_suite.py --config $arg --no-figures > $O/${T}_e2e_$arg.json 2> $O/${T}_e2e_$arg.err || exit $?; tail -1 $O/${T}_e2e_$arg.json ;;
    cpu)  # bench line with the multi-core C++ CPU baseline
      st=10; [ "$arg" != c2 ] && st=5
      timeout -k 10 900 python -u bench.py --config $arg --steps $st --warmup 2 > $O/${T}_cpu_$arg.json 2> $O/${T}_cpu_$arg.err || exit $?
      python3 -c "import json; d=json.loads([l for l in open('$O/${T}_cpu_$arg.json') if l.startswith('{')][-1]); print('$arg', d['ms_per_step'], d.get('cpu_baseline'), flush=True)" ;;
    fs|fs1)  # the sharded step at world 1 (fs1: its drivers in one host thread, fixed order)
      st=20; [ "$arg" != c2 ] && st=5
      extra=""; [ $kind = fs1 ] && extra="--shard-groups rq3,rq4b,rq2_count,rq1,rq4a,rq2_add"
      timeout -k 10 600 python -u bench.py --config $arg --steps $st --warmup 2 --no-cpu-baseline --probe-steps 0 --force-sharded $extra > $O/${T}_${kind}_$arg.json 2> $O/${T}_${kind}_$arg.err || exit $?
      python3 -c "import json; d=json.loads([l for l in open('$O/${T}_${kind}_$arg.json') if l.startswith('{')][-1]); print('$kind $arg', d['ms_per_step'], d['config'].get('driver_host_ms'), flush=True)" ;;
    profs)  # kernel trace of a serial step over some stages: profs:<cfg>@<stages>[@<shards of N: shard 0>]
      IFS=@ read -r cfg sts nsh <<< "$arg"
      nof=${nsh%%/*}; nrk=0; [ "$nsh" != "$nof" ] && nrk=${nsh#*/}  # N or N/rank
      extra=""; [ -n "$nsh" ] && extra="--strong --shard-of $nof --shard-rank $nrk"
      nsh=${nsh//\//_}
      timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/${T}_profs_$cfg$nsh -o run -- python3 -u bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --probe-steps 0 --serial --stages $sts $extra > $O/${T}_profs_$cfg$nsh.log 2>&1 || exit $?
      echo "profs $cfg $sts ok" ;;
    sho)  # sharded step (one rank) with a driver order: sho:<cfg>@<N>@<order>  (N = 0: the whole
          # table through --force-sharded; N > 0: shard 0 of N, --strong --force-sharded; order "x":
          # the default); sho:<cfg>@<N>@single: shard 0 of N through the single-table step
      IFS=@ read -r cfg n ord <<< "$arg"
      nr=0; [ "${n#*/}" != "$n" ] && nr=${n#*/} && n=${n%%/*}  # N or N/rank
      extra="--force-sharded"; [ "$n" != 0 ] && extra="$extra --strong --shard-of $n --shard-rank $nr"
      [ "$ord" = single ] && extra="--strong --shard-of $n --shard-rank $nr"
      [ "$ord" != x ] && [ "$ord" != single ] && extra="$extra --shard-groups $ord"
      st=20; [ "$cfg" != c2 ] && st=10
      timeout -k 10 400 python -u bench.py --config $cfg --steps $st --warmup 2 --no-cpu-baseline --probe-steps 0 $extra > $O/${T}_sho.json 2> $O/${T}_sho.err || exit $?
      python3 -c "import json; d=json.loads([l for l in open('$O/${T}_sho.json') if l.startswith('{')][-1]); print('sho $cfg $n $ord', d['ms_per_step'], d['config'].get('driver_host_ms'), flush=True)" ;;
    storeab)  # the store build with and without its helper fork (FZ_STORE_FORK), scripts/store_ab.sh
      CONFIG=$arg timeout -k 10 900 bash scripts/store_ab.sh > $O/${T}_storeab_$arg.txt 2>&1 || exit $?; cat $O/${T}_storeab_$arg.txt ;;
    ab)  # same-box A/B of library variants: ab:<name>+<name>... (base = lib/libfz.so), BENCH_ARGS
      VARIANTS="${arg//+/ }" timeout -k 10 900 bash scripts/bench_ab.sh > $O/${T}_ab.txt 2>&1 || exit $?; cat $O/${T}_ab.txt ;;
    envb)  # bench line under one runtime environment variable: envb:<cfg>@VAR=VALUE
      cfg=${arg%%@*}; kv=${arg#*@}; st=20; [ "$cfg" != c2 ] && st=5
      env "$kv" timeout -k 10 600 python -u bench.py --config $cfg --steps $st --warmup 2 --no-cpu-baseline > $O/${T}_envb.json 2> $O/${T}_envb.err || exit $?
      python3 -c "import json; d=json.loads([l for l in open('$O/${T}_envb.json') if l.startswith('{')][-1]); print('envb $cfg $kv', d['ms_per_step'], flush=True)" ;;
    fsprof)  # the sharded step at world 1 under cProfile (host time per function; pstats offline)
      timeout -k 10 600 python -u -m cProfile -o $O/${T}_fsprof_$arg.prof bench.py --config $arg --steps 100 --warmup 2 --no-cpu-baseline --probe-steps 0 --force-sharded > $O/${T}_fsprof_$arg.json 2> $O/${T}_fsprof_$arg.err || exit $?
      python3 -c "import pstats; pstats.Stats('$O/${T}_fsprof_$arg.prof').sort_stats('tottime').print_stats(25)" > $O/${T}_fsprof_$arg.txt && head -60 $O/${T}_fsprof_$arg.txt ;;
    sprobe)  # the store build's host vs GPU time
      timeout -k 10 300 python -u scripts/store_probe.py --config $arg > $O/${T}_sprobe_$arg.txt 2>&1 || exit $?
      grep '^{' $O/${T}_sprobe_$arg.txt ;;
    dmicro)  # describe-by-selection micro-benchmark (default build; phase stamps from the timing variant)
      timeout -k 10 200 python -u scripts/describe_micro.py > $O/${T}_dmicro.txt 2>&1 || exit $?
      V=tse-replication-package-1-million-fuzzing-sessions_amd/csrc/build/variants/libfz_desctime.so
      if [ -f $V ]; then TIMING=1 timeout -k 10 200 python -u scripts/describe_micro.py $V >> $O/${T}_dmicro.txt 2>&1 || exit $?; fi
      grep '^{' $O/${T}_dmicro.txt ;;
    grp)  # bench with another grouping of the analyses: grp:<cfg>@<groups> ("|" between streams)
      cfg=${arg%%@*}; groups=${arg#*@}
      timeout -k 10 600 python -u bench.py --config $cfg --steps 20 --warmup 2 --no-cpu-baseline --probe-steps 0 --groups "$groups" > $O/${T}_grp.json 2> $O/${T}_grp.err || exit $?
      python3 -c "import json; d=json.loads([l for l in open('$O/${T}_grp.json') if l.startswith('{')][-1]); print('grp $cfg $groups', d['ms_per_step'], flush=True)" ;;
    micro)  # radix micro-benchmark over library variants: micro:<v1>+<v2>... (SIZES, BITS, PROBE, KIND)
      timeout -k 10 400 python -u scripts/radix_micro.py ${arg//+/ } > $O/${T}_micro.txt 2>&1 || exit $?; cat $O/${T}_micro.txt ;;
    smicro)  # k_series_small micro-benchmark (default build, then the FZ_SERIES_TIMING variant sertime)
      timeout -k 10 200 python -u scripts/series_micro.py > $O/${T}_smicro.txt 2>&1 || exit $?
      for v in sertime sertimend; do
        V=tse-replication-package-1-million-fuzzing-sessions_amd/csrc/build/variants/libfz_$v.so
        if [ -f $V ]; then echo "# $v" >> $O/${T}_smicro.txt; timeout -k 10 200 python -u scripts/series_micro.py $V >> $O/${T}_smicro.txt 2>&1 || exit $?; fi
      done
      grep '^[{#]' $O/${T}_smicro.txt ;;
    tests)
      k=""; [ "$arg" != tests ] && k="${arg//+/ or }"
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread ${k:+-k "$k"} > $O/${T}_pytest.log 2>&1; rc=$?
      echo "pytest rc=$rc"; tail -3 $O/${T}_pytest.log; [ $rc -ne 0 ] && exit $rc ;;
  esac
done
echo done
