#!/bin/bash
# A/B of libgolhip variants on the GPU box: tools/ab.sh "<tune args>" variant...  (base = libgolhip.so)
set -e
ARGS=$1; shift
for v in "$@"; do
  if [ "$v" = base ]; then L=mpi_amd/libgolhip.so; else L=mpi_amd/libgolhip_$v.so; fi
  GOL_LIB=$L timeout -k 10 200 python tools/tune.py $ARGS | sed "s/^{/{\"v\":\"$v\",/" >> gpurun_out/ab.jsonl
done
