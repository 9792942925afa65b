# Round 5: RCCL-shim tests (split override mid-trial, config-5 seam windows) and the fuzz set with the split drawn.
set -e
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rccl_shim.py > gpurun_out/r05q_shim_tests.log 2>&1
tail -2 gpurun_out/r05q_shim_tests.log
bash tools/fuzz_set.sh r05q 521
