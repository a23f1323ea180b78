#!/bin/bash
# A/B of library variants on one box: VARIANTS="name ..." (build/variants/libfz_<name>.so; "base" = lib/libfz.so)
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out; mkdir -p $O
V=tse-replication-package-1-million-fuzzing-sessions_amd/csrc/build/variants
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-base}; do
    if [ "$v" = base ]; then lib=""; else lib=$PWD/$V/libfz_$v.so; fi
    FZ_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --steps 50 --warmup 3 --no-cpu-baseline --probe-steps 0 $BENCH_ARGS > $O/bab_${v}_$r.log 2>&1 || exit $?
    echo "$v $r $(grep -o '"ms_per_step": [0-9.]*' $O/bab_${v}_$r.log)"
  done
done
