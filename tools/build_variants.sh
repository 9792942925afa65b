#!/bin/bash
# Build A/B variants of libgolhip.so that differ only in compile-time kernel knobs.
# Select one at run time with GOL_LIB=<path>.
#   tools/build_variants.sh [name:flags ...]     (e.g. dppor:-DGOL_HSUM_DPP_OR=1)
set -euo pipefail
cd "$(dirname "$0")/../mpi_amd"
make -s -j4 libgolhip.so
mkdir -p build/variants
VARIANTS=("$@")
[ ${#VARIANTS[@]} -eq 0 ] && { echo "usage: tools/build_variants.sh name:flags ..."; exit 2; }
for v in "${VARIANTS[@]}"; do
  n=${v%%:*}; f=${v#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $f -c csrc/gol_kernels.hip -o build/variants/k_$n.o &
done
wait
for v in "${VARIANTS[@]}"; do
  n=${v%%:*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o libgolhip_$n.so build/variants/k_$n.o build/gol_text.o \
    build/gol_runtime.o build/glibc_jump.o -ldl
done
