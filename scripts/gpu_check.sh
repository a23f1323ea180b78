#!/bin/bash
# GPU session: parity tests, smoke, bench, rocprof kernel stats.  Each GPU step has its own time
# limit; a fault / abort / timeout (exit >= 124) ends the script, an ordinary test failure does not.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-r03}
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name exit $rc"; tail -5 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal step $name ($rc): stopping"; exit $rc; fi
  return $rc
}
STEPS=${STEPS:-tests,smoke,bench,prof}
[[ ",$STEPS," == *,tests,* ]] && run pytest_gpu 1100 python -u -m pytest tests -m gpu -v --timeout 900 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} $PYTEST_ARGS
[[ ",$STEPS," == *,smoke,* ]] && run smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()"
[[ ",$STEPS," == *,bench,* ]] && run bench 400 python -u bench.py
[[ ",$STEPS," == *,rehearse2,* ]] && run bench_rehearse2 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --no-cpu-baseline
# PMC passes: one counter group per run (FETCH_SIZE uses 3 TCC slots, WRITE_SIZE 2), SIGKILL limit
[[ ",$STEPS," == *,pmcF,* ]] && run pmc_fetch 150 timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_$TAG -o run -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline
[[ ",$STEPS," == *,pmcW,* ]] && run pmc_write 150 timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_$TAG -o run -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline
[[ ",$STEPS," == *,c3,* ]] && run bench_c3 600 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline
[[ ",$STEPS," == *,c3cpu,* ]] && run bench_c3_cpu 900 python -u bench.py --config c3 --steps 5 --warmup 2
[[ ",$STEPS," == *,c5cpu,* ]] && run bench_c5_cpu 900 python -u bench.py --config c5 --steps 5 --warmup 2
[[ ",$STEPS," == *,c4,* ]] && run bench_c4 300 python -u bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline
[[ ",$STEPS," == *,c5,* ]] && run bench_c5 600 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline
[[ ",$STEPS," == *,pc3,* ]] && run prof_c3 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3_$TAG -o run -- python -u bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline
[[ ",$STEPS," == *,pc5,* ]] && run prof_c5 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5_$TAG -o run -- python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline
[[ ",$STEPS," == *,fs2,* ]] && run bench_fs_c2 400 python -u bench.py --force-sharded --no-cpu-baseline
[[ ",$STEPS," == *,fs3,* ]] && run bench_fs_c3 600 python -u bench.py --config c3 --force-sharded --steps 3 --warmup 1 --no-cpu-baseline
[[ ",$STEPS," == *,strong3,* ]] && run bench_strong_c3 600 python -u bench.py --config c3 --strong --force-sharded --steps 3 --warmup 1 --no-cpu-baseline
[[ ",$STEPS," == *,e2e,* ]] && run e2e_c2 600 python -u scripts/e2e_suite.py --config c2
[[ ",$STEPS," == *,e2enofig,* ]] && run e2e_c2_nofig 600 python -u scripts/e2e_suite.py --config c2 --no-figures
[[ ",$STEPS," == *,prof,* ]] && run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline
echo done
