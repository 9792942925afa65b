set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
T=${1:-r04e}
timeout -k 10 600 python -u tools/fuzz.py --cases 300 --seed 401 --bit-k 8,3,5 > gpurun_out/${T}_fuzz_seed401_bitk8.log 2>&1
tail -1 gpurun_out/${T}_fuzz_seed401_bitk8.log
timeout -k 10 600 python -u tools/fuzz.py --cases 300 --seed 403 > gpurun_out/${T}_fuzz_seed403.log 2>&1
tail -1 gpurun_out/${T}_fuzz_seed403.log
timeout -k 10 600 python -u tools/fuzz.py --cases 120 --seed 405 --rccl-shim tests/shim/libfake_rccl.so > gpurun_out/${T}_fuzz_rccl_seed405.log 2>&1
tail -1 gpurun_out/${T}_fuzz_rccl_seed405.log
