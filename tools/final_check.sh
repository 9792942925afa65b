# GPU round check: the -m gpu suite, smoke and the driver's exact bench command.
#   bash tools/final_check.sh <tag>      (outputs under gpurun_out/<tag>_*)
set -e
T=${1:-check}
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${T}_gpu_tests.log 2>&1
tail -2 gpurun_out/${T}_gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
cat gpurun_out/${T}_smoke.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench_driver_cmd.json 2> gpurun_out/${T}_bench_driver_cmd.err
python3 -c "import json; d=json.load(open('gpurun_out/${T}_bench_driver_cmd.json')); print(d['value'], d['config']['chunk_policy'], d.get('clock',{}).get('sclk_mhz'), d['verified'], (d.get('aged_board') or {}).get('value'), (d.get('config4_1000gen') or {}).get('value'), {k: round(v.get('value', 0)) for k,v in d.get('secondary',{}).items()})"
