#!/bin/bash
# round-3 GPU session E: full GPU suite + smoke, then the round profiles (kernel stats + serial
# FETCH_SIZE / WRITE_SIZE passes) for c2 c3 c5
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=${TAG:-r3e}
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread > $O/${T}_pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 $O/${T}_pytest.log
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || exit $?
  echo smoke ok
fi
CONFIGS="${CONFIGS:-c2 c3 c5}" bash scripts/prof_round.sh || exit $?
