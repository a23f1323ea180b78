#!/bin/bash
# Build-log classification A/B on one box: the one-pass line scan (lib/libfz.so) vs the
# pattern-by-pattern variant (build/variants/libfz_bl0.so), scripts/bench_buildlog.py twice each.
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out; mkdir -p $O
V=tse-replication-package-1-million-fuzzing-sessions_amd/csrc/build/variants
for r in 1 2; do
  for v in base bl0; do
    lib=""; [ $v != base ] && lib=$PWD/$V/libfz_$v.so
    FZ_LIB_PATH=$lib timeout -k 10 300 python -u scripts/bench_buildlog.py > $O/bl_${v}_$r.json 2> $O/bl_${v}_$r.err || exit $?
    echo "$v $r $(tail -1 $O/bl_${v}_$r.json | cut -c1-400)"
  done
done
