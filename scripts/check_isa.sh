#!/bin/bash
# Emit the gfx950 device assembly of every libfz source and fail if any instruction writes
# through the scalar data cache (s_store*/s_buffer_store*/s_scratch_store*/scalar atomics/
# s_dcache_wb/s_dcache_discard) - the kernels only ever store through vector memory ops.
set -euo pipefail
cd "$(dirname "$0")/../tse-replication-package-1-million-fuzzing-sessions_amd/csrc"
out=$(mktemp -d)
for f in *.hip; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I../../include \
        --cuda-device-only -S "$f" -o "$out/${f%.hip}.s" 2>/dev/null &
done
wait
bad=$( (grep -hE "^\s+(s_store|s_buffer_store|s_scratch_store|s_dcache_wb|s_dcache_discard|s_atomic|s_buffer_atomic)" "$out"/*.s || true) | wc -l)
echo "device asm: $(cat "$out"/*.s | wc -l) lines, scalar-store instructions: $bad"
rm -rf "$out"
[ "$bad" -eq 0 ]
