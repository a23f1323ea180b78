#!/bin/bash
# GPU parity suite on the in-tree library, then the A/B bench of VARIANTS
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -1 $O/pytest_gpu.log; grep -E "FAILED" $O/pytest_gpu.log | head -5; [ $rc -ne 0 ] && exit $rc
bash scripts/bench_ab.sh
