# Round 5: interior split into 3 / 4 parts — parity, then tune.py at each part count.
set -e
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "split or k8_schedule or headline or uneven_gap" > gpurun_out/r05o_split_tests.log 2>&1
tail -2 gpurun_out/r05o_split_tests.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_runtime.py tests/test_gpu_rccl_shim.py > gpurun_out/r05o_rt_tests.log 2>&1
tail -2 gpurun_out/r05o_rt_tests.log
timeout -k 10 500 python tools/tune.py --spec 8:-2:2 --spec 8:-2:3 --spec 8:-1:3 --spec 8:-2:4 --spec 8:-1:4 --spec 8:-3:3 --spec 8:d:1 --gens 400 --reps 3 > gpurun_out/r05o_parts_tune.jsonl
cat gpurun_out/r05o_parts_tune.jsonl
