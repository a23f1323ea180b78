set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_rankstress.py tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo pytest $rc; tail -3 gpurun_out/pytest_gpu.log; grep -E "FAILED|float mismatch|^ours|^ref" gpurun_out/pytest_gpu.log | head -30
exit $rc
