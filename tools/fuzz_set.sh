#!/bin/bash
# The round's fuzz set on the GPU box (tools/fuzz.py against the oracle):
# every path, bit k = 8/3/5 heavy, the RCCL-mode transport over the shim, and real RCCL
# between rank processes on the one GPU (tests/rccl_real2_check.py --cases).
#   bash tools/fuzz_set.sh <tag> [seed0]      (logs under gpurun_out/<tag>_fuzz_*.log)
set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
T=${1:?tag}; S=${2:-411}
timeout -k 10 600 python -u tools/fuzz.py --cases 300 --seed $S --bit-k 8,3,5 > gpurun_out/${T}_fuzz_seedA_bitk8.log 2>&1
tail -1 gpurun_out/${T}_fuzz_seedA_bitk8.log
timeout -k 10 600 python -u tools/fuzz.py --cases 300 --seed $((S + 2)) > gpurun_out/${T}_fuzz_seedB.log 2>&1
tail -1 gpurun_out/${T}_fuzz_seedB.log
timeout -k 10 600 python -u tools/fuzz.py --cases 120 --seed $((S + 4)) --rccl-shim tests/shim/libfake_rccl.so \
  > gpurun_out/${T}_fuzz_rccl_seedC.log 2>&1
tail -1 gpurun_out/${T}_fuzz_rccl_seedC.log
timeout -k 10 900 python -u tests/rccl_real2_check.py --cases 20 --seed $((S + 6)) > gpurun_out/${T}_fuzz_rccl_real.log 2>&1
tail -1 gpurun_out/${T}_fuzz_rccl_real.log
