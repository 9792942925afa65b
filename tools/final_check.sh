set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03q_gpu_tests.log 2>&1
tail -2 gpurun_out/r03q_gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03q_smoke.log 2>&1
cat gpurun_out/r03q_smoke.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03q_bench_driver_cmd.json 2> gpurun_out/r03q_bench_driver_cmd.err
python3 -c "import json; d=json.load(open('gpurun_out/r03q_bench_driver_cmd.json')); print(d['value'], d['config']['chunk_policy'], d.get('clock',{}).get('sclk_mhz'), d['verified'], d.get('fresh_board',{}).get('value'), {k: round(v['value']) for k,v in d.get('secondary',{}).items()})"
