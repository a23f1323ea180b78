#!/bin/bash
# staged graph diagnostics, then the graph parity tests and the graph / no-graph bench
cd "$(dirname "$0")/.." || exit 1
STAGES="radix child;rq rq1 child tiny norebuild;rq rq3 child tiny rebuild;rq rq2_count parent tiny rebuild;rq rq4b child medium rebuild" bash scripts/graph_diag.sh || exit $?
bash scripts/gpu_graph_check.sh
