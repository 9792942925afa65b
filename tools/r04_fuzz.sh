set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
T=${1:-r04e}
timeout -k 10 600 python -u tools/fuzz.py --cases 300 --seed ${SEED0:-411} --bit-k 8,3,5 > gpurun_out/${T}_fuzz_seedA_bitk8.log 2>&1
tail -1 gpurun_out/${T}_fuzz_seedA_bitk8.log
timeout -k 10 600 python -u tools/fuzz.py --cases 300 --seed $(( ${SEED0:-411} + 2 )) > gpurun_out/${T}_fuzz_seedB.log 2>&1
tail -1 gpurun_out/${T}_fuzz_seedB.log
timeout -k 10 600 python -u tools/fuzz.py --cases 120 --seed $(( ${SEED0:-411} + 4 )) --rccl-shim tests/shim/libfake_rccl.so > gpurun_out/${T}_fuzz_rccl_seedC.log 2>&1
tail -1 gpurun_out/${T}_fuzz_rccl_seedC.log
