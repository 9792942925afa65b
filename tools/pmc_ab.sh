#!/bin/bash
set -euo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp; cd /tmp
for v in base old; do
  if [ $v = base ]; then L=$REPO/mpi_amd/libgolhip.so; else L=$REPO/mpi_amd/libgolhip_$v.so; fi
  for k in 7; do
    GOL_LIB=$L timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM \
      --output-format csv -d $OUT/pab_${v}_k$k -o run -- python3 $REPO/bench.py --no-cpu-baseline --no-secondary --steps 20 --warmup 2 -k $k > $OUT/pab_${v}_k$k.json 2>$OUT/pab_${v}_k$k.err
  done
done
echo ok
