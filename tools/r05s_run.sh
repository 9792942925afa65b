# Round 5: the schedule race check on the GPU (recorded schedules, happens-before).
set -e
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sched.py > gpurun_out/r05s_sched_tests.log 2>&1
tail -2 gpurun_out/r05s_sched_tests.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rccl_shim.py -k sched > gpurun_out/r05s_shim_sched.log 2>&1
tail -2 gpurun_out/r05s_shim_sched.log
