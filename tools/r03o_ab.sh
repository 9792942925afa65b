set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "chunk or k8" > gpurun_out/r03p_ts_tests.log 2>&1 || true
tail -2 gpurun_out/r03p_ts_tests.log
for r in 1 2; do timeout -k 10 400 python tools/tune.py --layout bit --gens 800 --reps 2 --spec 8:-6 --spec 8:-3 --spec 8:-1021 --spec 8:-1022 --spec 8:-1031 --spec 8:-1012 --spec 8:-1051 | sed "s/^{/{\"round\":$r,/" >> gpurun_out/r03p_tallshort.jsonl; done
cat gpurun_out/r03p_tallshort.jsonl
