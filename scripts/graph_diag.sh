#!/bin/bash
# Graph-recording diagnostics (scripts/graph_diag.py), one process per stage, stop at the first failure.
# STAGES: ';'-separated argument lists, e.g. "radix child;rq rq1 child tiny norebuild"
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O; : > $O/graph_diag.log
IFS=';' read -ra LIST <<< "${STAGES:-rq rq1 child tiny norebuild}"
for s in "${LIST[@]}"; do
  echo "== $s" >> $O/graph_diag.log
  timeout -k 10 120 python -u scripts/graph_diag.py $s >> $O/graph_diag.log 2>&1
  rc=$?; echo "$s rc=$rc"
  if [ $rc -ne 0 ]; then grep -v "^frame" $O/graph_diag.log | tail -40; exit $rc; fi
done
echo done
