set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo pytest $rc; tail -2 gpurun_out/pytest_gpu.log; grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -10
[ $rc -ne 0 ] && exit $rc
EXTRA=--force-sharded bash scripts/stage_times.sh
