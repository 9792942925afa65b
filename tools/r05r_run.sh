# Round 5: fixed cuts across block depths — split parity, then the fuzz set (seed 521 again: case 56).
set -e
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "split" > gpurun_out/r05r_split_tests.log 2>&1
tail -2 gpurun_out/r05r_split_tests.log
bash tools/fuzz_set.sh r05r 521
