#!/bin/bash
# Build libfz variants that differ only in compile-time tuning macros (radix tile shape, look-back
# window, sort block sizes, ...) for A/B runs on the GPU box (scripts/gpu_exp.sh, radix_micro.py).
# usage: scripts/build_variants.sh NAME "-DFZ_OS_BLOCK=512 ..." [NAME FLAGS ...]
set -euo pipefail
cd "$(dirname "$0")/../tse-replication-package-1-million-fuzzing-sessions_amd/csrc"
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I../../include -Wall -Wno-unused-function"
while [ $# -ge 2 ]; do
  name=$1; extra=$2; shift 2
  d=build/variants/$name
  mkdir -p $d
  for f in *.hip; do
    /opt/rocm/bin/hipcc $FLAGS $extra -c $f -o $d/${f%.hip}.o &
  done
  wait
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o build/variants/libfz_$name.so $d/*.o
  rm -rf $d
  echo "built build/variants/libfz_$name.so ($extra)"
done
