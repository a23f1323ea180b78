#!/bin/bash
# Build libfz variants that differ only in fz_prims.hip compile-time tuning macros (radix tile
# items per thread, look-back window) for the radix micro-benchmark (scripts/radix_micro.py).
# usage: scripts/build_variants.sh NAME "-DFZ_OS_ITEMS=8 -DFZ_OS_WINDOW=16" [NAME FLAGS ...]
set -euo pipefail
cd "$(dirname "$0")/../tse-replication-package-1-million-fuzzing-sessions_amd/csrc"
make -s -j8 >/dev/null
mkdir -p build/variants
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I../../include -Wall -Wno-unused-function"
while [ $# -ge 2 ]; do
  name=$1; extra=$2; shift 2
  /opt/rocm/bin/hipcc $FLAGS $extra -c fz_prims.hip -o build/variants/fz_prims_$name.o
  objs=$(ls build/*.o | grep -v fz_prims.o)
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o build/variants/libfz_$name.so $objs build/variants/fz_prims_$name.o
  echo "built build/variants/libfz_$name.so ($extra)"
done
