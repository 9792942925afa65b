# Round 5: the split interior (GOL_OPT_INTERIOR_SPLIT): parity, then a same-box sweep.
set -e
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "split" > gpurun_out/r05k_split_tests.log 2>&1
tail -1 gpurun_out/r05k_split_tests.log
timeout -k 10 400 python tools/tune.py --spec 8:d:1 --spec 8:d:2 --spec 8:-3:1 --spec 8:-3:2 --spec 8:-6:2 --spec 8:-2:2 --gens 400 --reps 3 > gpurun_out/r05k_split_tune.jsonl
cat gpurun_out/r05k_split_tune.jsonl
