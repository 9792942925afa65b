# Round 5: the 8-slab single-process rehearsal of config 5 (r05d: 104.9 k under a kernel
# trace, r03 137.7-139.1 k) without rocprof, per chunk policy, against one slab.
set -e
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rccl_shim.py tests/test_gpu_runtime.py > gpurun_out/r05e_tests.log 2>&1
tail -1 gpurun_out/r05e_tests.log
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
O=gpurun_out/r05e_sp8.jsonl
: > $O
for c in default -104 -6 -3; do
  A="--single-process --gpus 8 --no-secondary --no-cpu-baseline --steps 40 --warmup 5"
  [ "$c" != default ] && A="$A --chunk $c"
  timeout -k 10 300 python3 bench.py $A > /tmp/sp8.json 2> /tmp/sp8.err
  python3 -c "import json,sys; d=json.load(open('/tmp/sp8.json')); print(json.dumps({'chunk':sys.argv[1],'value':round(d['value']),'ms_per_step':round(d['ms_per_step'],3),'policy':d['config']['chunk_policy'],'mhz':(d.get('clock') or {}).get('sclk_mhz'),'verified':d['verified']}))" "$c" >> $O
  tail -1 $O
done
timeout -k 10 300 python3 bench.py --no-secondary --no-cpu-baseline --no-config4 --steps 40 --warmup 5 > /tmp/one.json
python3 -c "import json; d=json.load(open('/tmp/one.json')); print(json.dumps({'one_slab':round(d['value']),'policy':d['config']['chunk_policy'],'mhz':(d.get('clock') or {}).get('sclk_mhz')}))" >> $O
tail -1 $O
