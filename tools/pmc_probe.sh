#!/bin/bash
# Two PMC passes over tools/tune.py for one lib variant (run on the GPU box from the repo root):
#   tools/pmc_probe.sh <tag> <lib: base|name> "<tune.py args>"
set -u
TAG=$1; LIB=$2; ARGS=$3
R=$PWD
if [ "$LIB" = base ]; then L=$R/mpi_amd/libgolhip.so; else L=$R/mpi_amd/libgolhip_$LIB.so; fi
export TMPDIR=/tmp GOL_LIB=$L
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_IFETCH SQ_IFETCH_LEVEL SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE \
  --output-format csv -d $R/gpurun_out/pmc_${TAG}_a -o run -- python3 $R/tools/tune.py $ARGS > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_INSTS_SMEM SQ_BUSY_CU_CYCLES SQ_CYCLES \
  --output-format csv -d $R/gpurun_out/pmc_${TAG}_b -o run -- python3 $R/tools/tune.py $ARGS > /dev/null 2>&1 || exit 1
echo "pmc $TAG done"
