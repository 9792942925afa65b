#!/bin/bash
# Build A/B variants of libgolhip.so that differ only in compile-time kernel knobs
# (load/store cache policy).  Select one at run time with GOL_LIB=<path>.
set -euo pipefail
cd "$(dirname "$0")/../mpi_amd"
make -s -j4 libgolhip.so
mkdir -p build/variants
for v in "nts:-DGOL_STORE_AUX=2" "ntl:-DGOL_LOAD_AUX=2" "ntb:-DGOL_LOAD_AUX=2 -DGOL_STORE_AUX=2"; do
  n=${v%%:*}; f=${v#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $f -c csrc/gol_kernels.hip -o build/variants/k_$n.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o libgolhip_$n.so build/variants/k_$n.o build/gol_runtime.o build/glibc_jump.o -ldl
done
