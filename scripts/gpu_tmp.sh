set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo pytest $rc; tail -2 gpurun_out/pytest_gpu.log; grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -10
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_1.log 2>&1 || exit $?; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_1.log; done
