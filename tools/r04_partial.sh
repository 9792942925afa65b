set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_runtime.py tests/test_gpu_rccl_shim.py > gpurun_out/r04b_gpu_tests.log 2>&1
tail -2 gpurun_out/r04b_gpu_tests.log
