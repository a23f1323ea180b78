#!/bin/bash
# describe micro-benchmark per library variant (VARIANTS="base name ..."; build/variants/libfz_<name>.so)
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out; mkdir -p $O
V=tse-replication-package-1-million-fuzzing-sessions_amd/csrc/build/variants
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then lib=""; else lib=$PWD/$V/libfz_$v.so; fi
  echo "== $v"
  timeout -k 10 200 python -u scripts/describe_micro.py $lib 2>&1 | grep -v amdgpu.ids || exit $?
done
