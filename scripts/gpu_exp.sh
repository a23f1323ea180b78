# A/B experiment on the GPU box: radix micro-benchmark + bench per libfz variant, then the GPU tests.
set -o pipefail
V=tse-replication-package-1-million-fuzzing-sessions_amd/csrc/build/variants
VARIANTS=${VARIANTS:-old new}
[ -n "$NOMICRO" ] || timeout -k 10 200 python -u scripts/radix_micro.py $VARIANTS > gpurun_out/radix_micro.log 2>&1 || exit $?
if [ -f $V/libfz_timing.so ]; then TIMING=timing timeout -k 10 100 python -u scripts/radix_micro.py >> gpurun_out/radix_micro.log 2>&1 || exit $?; fi
for v in $VARIANTS; do
  FZ_LIB_PATH=$PWD/$V/libfz_$v.so timeout -k 10 200 python -u bench.py --no-cpu-baseline $BENCH_ARGS > gpurun_out/bench_$v.log 2>&1 || exit $?
done
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo pytest $?
grep -v amdgpu.ids gpurun_out/radix_micro.log
for v in $VARIANTS; do echo $v; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_$v.log; grep -o '"avg_launch_us": [0-9.]*' gpurun_out/bench_$v.log; done
tail -2 gpurun_out/pytest_gpu.log
