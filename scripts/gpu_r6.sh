#!/bin/bash
# Round-6 GPU steps.  STEPS: any of "full" (test_gpu_fullsize on K), "tests" (pytest TESTS),
# "bench" (bench.py on each of BENCH configs, with the CPU baseline), "strong" (strong rehearsal of
# CONFIG at NS shards, every shard).  Each step under its own time limit; the first failure ends it.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=${TAG:-r6}
for s in ${STEPS:-full bench}; do
  case $s in
    full)
      timeout -k 10 ${FULL_S:-800} python -u -m pytest tests/test_gpu_fullsize.py -k "${K:-c3L or c5L}" -m gpu -x -v -s \
        --timeout 900 --timeout-method thread > $O/${T}_full.log 2>&1
      rc=$?; echo "full rc $rc"; tail -2 $O/${T}_full.log; [ $rc -ne 0 ] && exit $rc ;;
    tests)
      timeout -k 10 ${TESTS_S:-800} python -u -m pytest $TESTS -m gpu -x -v -s --timeout 600 --timeout-method thread \
        > $O/${T}_tests.log 2>&1
      rc=$?; echo "tests rc $rc"; tail -2 $O/${T}_tests.log; [ $rc -ne 0 ] && exit $rc ;;
    bench)
      for c in ${BENCH:-c3L c5L c4}; do
        st=10; [ $c = c2 ] && st=20
        timeout -k 10 ${BENCH_S:-400} python -u bench.py --config $c --steps $st --warmup 2 $BENCH_ARGS \
          > $O/${T}_bench_$c.json 2> $O/${T}_bench_$c.err
        rc=$?; echo "bench $c rc $rc $(grep -o '"ms_per_step": [0-9.]*' $O/${T}_bench_$c.json | head -1)"
        [ $rc -ne 0 ] && { tail -5 $O/${T}_bench_$c.err; exit $rc; }
      done ;;
    prof)
      for c in ${PROF:-c5L}; do
        timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_$c -o run -- python3 -u bench.py \
          --config $c --steps 3 --warmup 1 --no-cpu-baseline --probe-steps 0 $PROF_ARGS > $O/${T}_prof_$c.log 2>&1
        rc=$?; echo "prof $c rc $rc"; [ $rc -ne 0 ] && { tail -5 $O/${T}_prof_$c.log; exit $rc; }
        python3 scripts/kstats.py $(find $O/${T}_prof_$c -name '*kernel_stats.csv' | head -1) auto 40 > $O/${T}_kstats_$c.txt
        head -25 $O/${T}_kstats_$c.txt
      done ;;
    ab)  # same-box A/B: ABSETS = bench argument sets separated by ';' (e.g. " ;--lanes 2"), ROUNDS rounds
      IFS=';' read -ra SETS <<< "${ABSETS:- }"
      for r in $(seq 1 ${ROUNDS:-2}); do
        for i in "${!SETS[@]}"; do
          a="${SETS[$i]}"
          # (a set may start with VAR=value words: the environment of that run, e.g. FZ_LIB_PATH=...)
          envs=(); args=()
          for w in $a; do if [[ ${#args[@]} -eq 0 && $w == *=* && $w != -* ]]; then envs+=("$w"); else args+=("$w"); fi; done
          timeout -k 10 300 env "${envs[@]}" python -u bench.py --config ${ABCONF:-c2} --steps ${ABSTEPS:-50} --warmup 3 --no-cpu-baseline \
            --probe-steps 0 "${args[@]}" > $O/${T}_ab_${i}_$r.log 2>&1 || { tail -5 $O/${T}_ab_${i}_$r.log; exit 1; }
          echo "ab[$i] '$a' r$r $(grep -o '"ms_per_step": [0-9.]*' $O/${T}_ab_${i}_$r.log)" | tee -a $O/${T}_ab.txt
        done
      done ;;
    strong)
      C=${CONFIG:-c3L}
      for n in ${NS:-1 8}; do
        for r in $(seq 0 $((n - 1))); do
          # (REPS runs per shard, each line kept; the summary takes each shard's fastest: one run can
          # land on a slow moment of the box)
          for k in $(seq 1 ${REPS:-1}); do
          timeout -k 10 300 python -u bench.py --config $C --steps 10 --warmup 2 --no-cpu-baseline --probe-steps 0 \
            --strong --force-sharded --shard-of $n --shard-rank $r > $O/${T}_sr.json 2> $O/${T}_sr.err || { tail -5 $O/${T}_sr.err; exit 1; }
          python3 -c "import json; d=json.loads([l for l in open('$O/${T}_sr.json') if l.startswith('{')][-1]); print('$C shard $r of $n', d['ms_per_step'], d['config']['rows_per_rank'], flush=True)" | tee -a $O/${T}_strong_$C.txt
          done
        done
      done ;;
  esac
done
echo done
